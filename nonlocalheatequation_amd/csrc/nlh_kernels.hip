// nlh_kernels.hip -- fp64 gfx950 kernels for the explicit-Euler step of the 2D
// nonlocal heat equation.
//
// Hot path replaced (reference /root/reference):
//   sum_local       src/2d_nonlocal_serial.cpp:256-270   (also async :364-379,
//                   distributed :1102-1117)
//   sum_local_test  src/2d_nonlocal_serial.cpp:235-252
//   do_work update  src/2d_nonlocal_serial.cpp:279-284
//   compute_l2/linf src/2d_nonlocal_serial.cpp:96-113
//
// Two stencil implementations share one launch interface (RectList):
//
//  k_exact  -- parity kernel.  One thread per node; the disk loop, the
//     per-term order ((c*(u_j-u_i))*dh^2) and the two separate roundings of
//     the update are the reference's, with FMA contraction disabled.  Bitwise
//     equal to the reference (w from host-computed glibc sin/cos tables).
//
//  k_fast   -- production kernel for J == 1 (influence_function, :201).  The
//     disk sum  S(x,y) = sum_{dx^2+dy^2<=E^2} u(x+dx,y+dy)  is evaluated by
//     nested row windows: for each input row r the lane forms
//        H_L(x,r) = sum_{|dx|<=L} u(x+dx,r),  L = 0..E  (2 adds per level)
//     and scatters H_{len(dy)}(x,r) into the 2E+1 register accumulators of
//     the outputs y = r-dy.  ~4E+1 adds per node instead of N(E) (197 at
//     E=8) -> the kernel is HBM-bound.  Update u' = u + (S - N u)*c*dh^2*dt.
//     One wave sweeps a strip of 64*R columns down a segment of rows; rows
//     stream HBM -> LDS ring by LDS-DMA (global_load_lds_dwordx4) D rows
//     ahead, with hand-counted vmcnt waits (inline asm, so the compiler does
//     not drain the ring before every ds_read).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "nlh_fast.h"
#include "nlh_pair.h"
#include "nlh_wide.h"
#include "nlh_kernel_common.h"

namespace nlh {


// ----------------------------------------------------------------------------
// k_exact: bit-parity kernel.  64x4 nodes per 256-thread workgroup.
template <bool TEST, bool SUMONLY, bool WT>
__global__ __launch_bounds__(256) void k_exact(RectList L, StepConst C) {
#pragma clang fp contract(off)
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &R = L.r[ri];
  const int local = work - R.wg_begin;
  const int tx = local % R.nstrip, ty = local / R.nstrip;
  const int x = R.x0 + tx * 64 + (int)(threadIdx.x & 63);
  const int y = R.y0 + ty * 4 + (int)(threadIdx.x >> 6);
  if (x >= R.x1 || y >= R.y1) return;
  const int64_t p = R.pitch;
  const int E = C.E;
  const double *u = R.u + (int64_t)y * p + x;
  const double ui = *u;
  double res = 0.0;
  // sum_local (:256-270): sx outer, sy inner; out-of-domain halo cells are 0.
  // The reference's term is ((J*c)*(u_j-u_i))*(dh*dh) with J = 1.0 (:201);
  // WT: J*c per disk point from the host table, same order
  if constexpr (WT) {
    int n = 0;
    for (int dx = -E; dx <= E; ++dx) {
      const int len = C.lens[dx < 0 ? -dx : dx];
      const double *col = u + dx;
      for (int dy = -len; dy <= len; ++dy, ++n)
        res += ((C.wt[n] * (col[(int64_t)dy * p] - ui)) * C.dh2);
    }
  } else {
    for (int dx = -E; dx <= E; ++dx) {
      const int len = C.lens[dx < 0 ? -dx : dx];
      const double *col = u + dx;
      for (int dy = -len; dy <= len; ++dy)
        res += ((C.c2d * (col[(int64_t)dy * p] - ui)) * C.dh2);
    }
  }
  if (SUMONLY) {
    R.un[(int64_t)y * p + x] = res;
    return;
  }
  double out = ui + (res * C.dt);
  if (TEST) {
    // sum_local_test (:235-252) with w = (cos*sin(x))*sin(y) from tables
    const int gx = R.gx0 + x, gy = R.gy0 + y;
    const double sxv = C.sxt[gx + E], syv = C.syt[gy + E];
    double r2 = -((C.st2pi * sxv) * syv);
    const double wpos = (C.ct * sxv) * syv;
    int n = 0;
    for (int dx = -E; dx <= E; ++dx) {
      const int len = C.lens[dx < 0 ? -dx : dx];
      const int sx = gx + dx;
      const bool inx = (sx >= 0) && (sx < C.nx);
      const double cx = C.ct * C.sxt[sx + E];
      for (int dy = -len; dy <= len; ++dy, ++n) {
        const int sy = gy + dy;
        const bool in = inx && (sy >= 0) && (sy < C.ny);
        const double wv = in ? (cx * C.syt[sy + E]) : 0.0;
        r2 -= (((WT ? C.wt[n] : C.c2d) * (wv - wpos)) * C.dh2);
      }
    }
    out += r2 * C.dt;
  }
  R.un[(int64_t)y * p + x] = out;
}

// ----------------------------------------------------------------------------
// k_exact_lds: the bit-parity kernel with the lattice staged in LDS.  A
// 256-thread workgroup owns 64 x 16 nodes; its (64+2E) x (16+2E) tile of u
// (and in test mode of w = (ct*sin x)*sin y, 0 outside the domain: the value
// k_exact forms per term, formed once here) sits in LDS.  Each thread runs 4
// vertically adjacent nodes of one column through the reference's loop
// (sx outer, sy inner; ((J*c)*(u_j-u_i))*dh^2 accumulated in order, no FMA
// contraction), so for every (dx, dy) the 4 nodes read 4 consecutive tile
// rows: a 4-value register window slides down the column, one LDS read per
// term per 4 nodes.  Bitwise equal to k_exact.
template <bool TEST, bool WT>
__global__ __launch_bounds__(256) void k_exact_lds(RectList L, StepConst C) {
#pragma clang fp contract(off)
  extern __shared__ double tile[];
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &R = L.r[ri];
  const int local = work - R.wg_begin;
  const int tx = local % R.nstrip, ty = local / R.nstrip;
  const int E = C.E;
  const int x0 = R.x0 + tx * 64, y0 = R.y0 + ty * 16;
  const int TW = 64 + 2 * E, TH = 16 + 2 * E;
  const int64_t p = R.pitch;
  const int ylast = R.y1 + E - 1;  // rows past it only feed nodes that are not stored
  double *wtile = tile + TW * TH;
  for (int e = (int)threadIdx.x; e < TW * TH; e += 256) {
    const int r = e / TW, cc = e - r * TW;
    const int gy = min(y0 - E + r, ylast);
    tile[e] = R.u[(int64_t)gy * p + (x0 - E + cc)];
    if (TEST) {
      const int sx = R.gx0 + x0 - E + cc, sy = R.gy0 + y0 - E + r;
      const bool in = sx >= 0 && sx < C.nx && sy >= 0 && sy < C.ny;
      wtile[e] = in ? (C.ct * C.sxt[sx + E]) * C.syt[sy + E] : 0.0;
    }
  }
  __syncthreads();
  const int lx = (int)(threadIdx.x & 63), ly = (int)(threadIdx.x >> 6) * 4;
  const int x = x0 + lx;
  const double *c = tile + (ly + E) * TW + (lx + E);  // node (x, y0 + ly)
  double ui[4], res[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 4; ++k) ui[k] = c[k * TW];
  const double c2d = C.c2d, dh2 = C.dh2;
  // one disk column: 4 nodes, terms in the reference's dy order each; four dy
  // per iteration so the window slides by renaming (3 moves per 4 dy) and the
  // 4 LDS reads of a block are in flight together
  auto column = [&](const double *col, int len, int n, double (&acc)[4], const double (&ref)[4],
                    bool sub) __attribute__((always_inline)) {
    double v0 = col[-len * TW], v1 = col[(1 - len) * TW], v2 = col[(2 - len) * TW];
    auto term = [&](double &a, double wv, double v, double r) __attribute__((always_inline)) {
      if (sub)
        a -= ((wv * (v - r)) * dh2);
      else
        a += ((wv * (v - r)) * dh2);
    };
    int dy = -len;
    for (; dy + 3 <= len; dy += 4, n += 4) {
      const double v3 = col[(dy + 3) * TW], v4 = col[(dy + 4) * TW], v5 = col[(dy + 5) * TW],
                   v6 = col[(dy + 6) * TW];
      const double w0 = WT ? C.wt[n] : c2d, w1 = WT ? C.wt[n + 1] : c2d, w2 = WT ? C.wt[n + 2] : c2d,
                   w3 = WT ? C.wt[n + 3] : c2d;
      term(acc[0], w0, v0, ref[0]); term(acc[1], w0, v1, ref[1]); term(acc[2], w0, v2, ref[2]); term(acc[3], w0, v3, ref[3]);
      term(acc[0], w1, v1, ref[0]); term(acc[1], w1, v2, ref[1]); term(acc[2], w1, v3, ref[2]); term(acc[3], w1, v4, ref[3]);
      term(acc[0], w2, v2, ref[0]); term(acc[1], w2, v3, ref[1]); term(acc[2], w2, v4, ref[2]); term(acc[3], w2, v5, ref[3]);
      term(acc[0], w3, v3, ref[0]); term(acc[1], w3, v4, ref[1]); term(acc[2], w3, v5, ref[2]); term(acc[3], w3, v6, ref[3]);
      v0 = v4;
      v1 = v5;
      v2 = v6;
    }
    for (; dy <= len; ++dy, ++n) {
      const double v3 = col[(dy + 3) * TW];
      const double wv = WT ? C.wt[n] : c2d;
      term(acc[0], wv, v0, ref[0]); term(acc[1], wv, v1, ref[1]); term(acc[2], wv, v2, ref[2]); term(acc[3], wv, v3, ref[3]);
      v0 = v1;
      v1 = v2;
      v2 = v3;
    }
  };
  int n = 0;
  for (int dx = -E; dx <= E; ++dx) {
    const int len = C.lens[dx < 0 ? -dx : dx];
    column(c + dx, len, n, res, ui, false);
    n += 2 * len + 1;
  }
  double r2[4], wpos[4];
  if (TEST) {
    const int gx = min(R.gx0 + x, C.nx - 1);  // columns past the lattice: not stored
    const double sxv = C.sxt[gx + E];
    const double *cw = wtile + (ly + E) * TW + (lx + E);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // rows past the lattice only feed nodes that are not stored: clamp the
      // table index, keep the arithmetic
      const int gy = min(R.gy0 + y0 + ly + k, C.ny - 1);
      const double syv = C.syt[gy + E];
      r2[k] = -((C.st2pi * sxv) * syv);
      wpos[k] = (C.ct * sxv) * syv;
    }
    n = 0;
    for (int dx = -E; dx <= E; ++dx) {
      const int len = C.lens[dx < 0 ? -dx : dx];
      column(cw + dx, len, n, r2, wpos, true);
      n += 2 * len + 1;
    }
  }
  if (x >= R.x1) return;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int y = y0 + ly + k;
    if (y >= R.y1) break;
    double out = ui[k] + (res[k] * C.dt);
    if (TEST) out += r2[k] * C.dt;
    R.un[(int64_t)y * p + x] = out;
  }
}

// ----------------------------------------------------------------------------
// k_weighted: fast path for a non-constant radial J (influence != 0), and for
// J = 1 beyond the nested-window kernels' horizons (eps 33..52).  The
// nested-window kernels need J = 1; here each 256-thread workgroup stages a
// (64+2E) x (16+2E) tile of u in LDS (rows past the block clamp to its last
// halo row; they only feed outputs that are not stored) and each thread
// computes 4 outputs of one column:
//   S = J00 u + sum_{groups} J(dx,dy) * (sum of the <= 4 mirror points)
// (the disk |dy| <= len(|dx|) is symmetric in the signs of dx and dy), then
// u' = u + alpha (S - Jsum u)  [+ dt b in test mode, b from L_h^J[W0]].
template <bool TEST>
__global__ __launch_bounds__(256) void k_weighted(RectList L, StepConst C) {
  extern __shared__ double tile[];
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &R = L.r[ri];
  const int local = work - R.wg_begin;
  const int tx = local % R.nstrip, ty = local / R.nstrip;
  const int E = C.E;
  const int x0 = R.x0 + tx * 64, y0 = R.y0 + ty * 16;
  const int TW = 64 + 2 * E, TH = 16 + 2 * E;
  const int64_t p = R.pitch;
  // the block's allocation holds rows -E .. R.y1 + E - 1 of every rect in it
  const int ylast = R.y1 + E - 1;
  for (int e = (int)threadIdx.x; e < TW * TH; e += 256) {
    const int r = e / TW, cc = e - r * TW;
    const int gy = min(y0 - E + r, ylast);
    tile[e] = R.u[(int64_t)gy * p + (x0 - E + cc)];
  }
  __syncthreads();
  const int lx = (int)(threadIdx.x & 63), ly = (int)(threadIdx.x >> 6);
  const int x = x0 + lx;
  const double alpha = C.alpha, jsum = C.jsum;
  const int EW = E + 1;
  for (int k = 0; k < 4; ++k) {
    const int oy = ly + 4 * k;
    const int y = y0 + oy;
    if (x >= R.x1 || y >= R.y1) continue;
    const double *c = tile + (oy + E) * TW + (lx + E);
    const double uc = c[0];
    double s = C.qj[0] * uc;
    for (int dx = 1; dx <= E; ++dx) s = fma(C.qj[dx * EW], c[dx] + c[-dx], s);
    for (int dy = 1; dy <= E; ++dy) s = fma(C.qj[dy], c[dy * TW] + c[-dy * TW], s);
    for (int dx = 1; dx <= E; ++dx) {
      const int len = C.lens[dx];
      for (int dy = 1; dy <= len; ++dy) {
        const double *a = c + dy * TW, *b = c - dy * TW;
        s = fma(C.qj[dx * EW + dy], (a[dx] + a[-dx]) + (b[dx] + b[-dx]), s);
      }
    }
    double out = fma(alpha, fma(-jsum, uc, s), uc);
    if (TEST) {
      const int gx = R.gx0 + x, gyy = R.gy0 + y;
      const double w0 = C.sxt[gx + E] * C.syt[gyy + E];
      const double bsrc = -(C.st2pi * w0) - C.ct * R.lw[(int64_t)y * p + x];
      out = fma(bsrc, C.dt, out);
    }
    R.un[(int64_t)y * p + x] = out;
  }
}

// ----------------------------------------------------------------------------
// k_weighted_col: k_weighted's operator with the disk walked column by column
// (dx outer, dy inner) over the same LDS tile, J(dx, |dy|) staged in LDS too.
// Each thread owns 4 vertically adjacent nodes of one column; per dx > 0 the
// mirror columns are summed once per tile row, p(r) = u(x+dx, r) + u(x-dx, r),
// and a 4-value window of p slides down the column, so one pair of LDS reads
// and one add serve a row of 4 FMAs (k_weighted: 4 reads and 3 adds per group
// per node).  FMA order differs from k_weighted's: fast-mode tolerance.
template <bool TEST>
__global__ __launch_bounds__(256) void k_weighted_col(RectList L, StepConst C) {
  extern __shared__ double tile[];
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &R = L.r[ri];
  const int local = work - R.wg_begin;
  const int tx = local % R.nstrip, ty = local / R.nstrip;
  const int E = C.E;
  const int x0 = R.x0 + tx * 64, y0 = R.y0 + ty * 16;
  const int TW = 64 + 2 * E, TH = 16 + 2 * E;
  const int64_t p = R.pitch;
  const int ylast = R.y1 + E - 1;  // rows past it only feed nodes that are not stored
  double *qjs = tile + TW * TH;    // J(dx, dy), dx, dy in [0, E]
  for (int e = (int)threadIdx.x; e < TW * TH; e += 256) {
    const int r = e / TW, cc = e - r * TW;
    const int gy = min(y0 - E + r, ylast);
    tile[e] = R.u[(int64_t)gy * p + (x0 - E + cc)];
  }
  for (int e = (int)threadIdx.x; e < (E + 1) * (E + 1); e += 256) qjs[e] = C.qj[e];
  __syncthreads();
  const int lx = (int)(threadIdx.x & 63), ly = (int)(threadIdx.x >> 6) * 4;
  const double *c = tile + (ly + E) * TW + (lx + E);  // node (x0 + lx, y0 + ly)
  double sacc[4] = {0.0, 0.0, 0.0, 0.0};
  // one disk column pair: rows -len .. len+3 around the 4 nodes, four dy per
  // iteration (the window slides by renaming)
  auto column = [&](const double *a, const double *b, bool pair, int len, const double *jr)
      __attribute__((always_inline)) {
    auto pv = [&](int r) __attribute__((always_inline)) {
      return pair ? a[r * TW] + b[r * TW] : a[r * TW];
    };
    double v0 = pv(-len), v1 = pv(1 - len), v2 = pv(2 - len);
    int dy = -len;
    for (; dy + 3 <= len; dy += 4) {
      const double v3 = pv(dy + 3), v4 = pv(dy + 4), v5 = pv(dy + 5), v6 = pv(dy + 6);
      const double j0 = jr[abs(dy)], j1 = jr[abs(dy + 1)], j2 = jr[abs(dy + 2)], j3 = jr[abs(dy + 3)];
      sacc[0] = fma(j0, v0, sacc[0]); sacc[1] = fma(j0, v1, sacc[1]); sacc[2] = fma(j0, v2, sacc[2]); sacc[3] = fma(j0, v3, sacc[3]);
      sacc[0] = fma(j1, v1, sacc[0]); sacc[1] = fma(j1, v2, sacc[1]); sacc[2] = fma(j1, v3, sacc[2]); sacc[3] = fma(j1, v4, sacc[3]);
      sacc[0] = fma(j2, v2, sacc[0]); sacc[1] = fma(j2, v3, sacc[1]); sacc[2] = fma(j2, v4, sacc[2]); sacc[3] = fma(j2, v5, sacc[3]);
      sacc[0] = fma(j3, v3, sacc[0]); sacc[1] = fma(j3, v4, sacc[1]); sacc[2] = fma(j3, v5, sacc[2]); sacc[3] = fma(j3, v6, sacc[3]);
      v0 = v4;
      v1 = v5;
      v2 = v6;
    }
    for (; dy <= len; ++dy) {
      const double v3 = pv(dy + 3);
      const double j = jr[abs(dy)];
      sacc[0] = fma(j, v0, sacc[0]); sacc[1] = fma(j, v1, sacc[1]); sacc[2] = fma(j, v2, sacc[2]); sacc[3] = fma(j, v3, sacc[3]);
      v0 = v1;
      v1 = v2;
      v2 = v3;
    }
  };
  column(c, c, false, E, qjs);  // dx = 0 (len(0) = E)
  for (int dx = 1; dx <= E; ++dx) column(c + dx, c - dx, true, C.lens[dx], qjs + dx * (E + 1));
  const int x = x0 + lx;
  if (x >= R.x1) return;
  const double alpha = C.alpha, jsum = C.jsum;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int y = y0 + ly + k;
    if (y >= R.y1) break;
    const double uc = c[k * TW];
    double out = fma(alpha, fma(-jsum, uc, sacc[k]), uc);
    if (TEST) {
      const double w0 = C.sxt[R.gx0 + x + E] * C.syt[R.gy0 + y + E];
      const double bsrc = -(C.st2pi * w0) - C.ct * R.lw[(int64_t)y * p + x];
      out = fma(bsrc, C.dt, out);
    }
    R.un[(int64_t)y * p + x] = out;
  }
}

// ----------------------------------------------------------------------------
// 1D solver (src/1d_nonlocal_serial.cpp): one thread per node, the
// reference's per-term order; u has eps zero nodes on each side
template <bool TEST>
__global__ __launch_bounds__(256) void k_1d(const double *u, double *un, int64_t nx, int eps, double c,
                                            double dt, double dx, double st2pi, double ct,
                                            const double *sxt) {
#pragma clang fp contract(off)
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= nx) return;
  const double ui = u[x];
  double res = 0.0;  // sum_local (1d :198-206)
  for (int d = -eps; d <= eps; ++d) res += ((1.0 * c) * (u[x + d] - ui)) * dx;
  double out = ui + (res * dt);
  if (TEST) {  // sum_local_test (1d :186-195), w from the host sin table
    double r2 = -(st2pi * sxt[x + eps]);
    const double wpos = ct * sxt[x + eps];
    for (int d = -eps; d <= eps; ++d) {
      const int64_t sx = x + d;
      const double wv = (sx >= 0 && sx < nx) ? ct * sxt[sx + eps] : 0.0;
      r2 -= ((1.0 * c) * (wv - wpos)) * dx;
    }
    out += r2 * dt;
  }
  un[x] = out;
}

// compute_l2 / compute_linf (1d :91-103) in the reference's sequential order
// (one thread; the 1D lattices are small)
__global__ void k_1d_norms(const double *u, int64_t nx, int eps, double ct, const double *sxt,
                           double *out) {
#pragma clang fp contract(off)
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  double e2 = 0.0, ei = 0.0;
  for (int64_t x = 0; x < nx; ++x) {
    const double d = u[x] - ct * sxt[x + eps];
    e2 += d * d;
    ei = fmax(fabs(d), ei);
  }
  out[0] = e2;
  out[1] = ei;
}

int launch_1d(const double *u, double *un, int64_t nx, int32_t eps, double c1d, double dt, double dx,
              bool test, double st2pi, double ct, const double *sxt, void *stream) {
  const dim3 grid((unsigned)((nx + 255) / 256));
  if (test)
    hipLaunchKernelGGL(k_1d<true>, grid, dim3(256), 0, (hipStream_t)stream, u, un, nx, eps, c1d, dt, dx,
                       st2pi, ct, sxt);
  else
    hipLaunchKernelGGL(k_1d<false>, grid, dim3(256), 0, (hipStream_t)stream, u, un, nx, eps, c1d, dt, dx,
                       st2pi, ct, sxt);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int launch_1d_norms(const double *u, int64_t nx, int32_t eps, double ct, const double *sxt, double *out,
                    void *stream) {
  hipLaunchKernelGGL(k_1d_norms, dim3(1), dim3(64), 0, (hipStream_t)stream, u, nx, eps, ct, sxt, out);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// ----------------------------------------------------------------------------
// halo copies
__global__ __launch_bounds__(256) void k_copies(CopyList L) {
  const int work = blockIdx.x;
  int ci = 0;
  for (int k = 1; k < L.ncopies; ++k) ci = (work >= L.c[k].wg_begin) ? k : ci;
  const Copy &c = L.c[ci];
  const int64_t e = (int64_t)(work - c.wg_begin) * 256 + threadIdx.x;
  if (e >= (int64_t)c.w * c.h) return;
  const int64_t x = e % c.w, y = e / c.w;
  c.dst[y * c.dpitch + x] = c.src[y * c.spitch + x];
}

// test_init (:190-198) on the interior of a block
__global__ __launch_bounds__(256) void k_init_test(double *u, int64_t pitch,
                                                   int bx, int by, int gx0,
                                                   int gy0, StepConst C) {
#pragma clang fp contract(off)
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)bx * by) return;
  const int x = (int)(e % bx), y = (int)(e / bx);
  u[(int64_t)y * pitch + x] = C.sxt[gx0 + x + C.E] * C.syt[gy0 + y + C.E];
}

// W0 over the whole padded block (halo included), 0 outside the domain
__global__ __launch_bounds__(256) void k_fill_w0(double *u, int64_t pitch,
                                                 int xl, int rows, int halo, int gx0,
                                                 int gy0, StepConst C) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= pitch * rows) return;
  const int px = (int)(e % pitch), py = (int)(e / pitch);
  const int gx = gx0 + px - xl, gy = gy0 + py - halo;
  const bool in = gx >= 0 && gx < C.nx && gy >= 0 && gy < C.ny;
  u[e] = in ? C.sxt[gx + C.E] * C.syt[gy + C.E] : 0.0;
}

// L_h[W0] of the fast test mode from its separable form (compute_lw, J = 1;
// the tables of nlh_api.cpp sep_tables, long double on the host, c dh^2 in
// lsx): per node c dh^2 (sum_l Sx'_l(x) Ty_l(y) + sx(x) Z(y)) -- the
// reference's sum_local_test disk sum of W0 (:235-252) without its N(eps)
// sequential roundings, in the operation order of k_pair_split's SEP rows.
// Over the block-relative rectangle x0 .. x0+w, y0 .. y0+h (the block and the
// two-step kernel's frame), 0 outside the lattice; one thread per node
__global__ __launch_bounds__(256) void k_lw_sep(double *out, int64_t pitch, int x0, int y0, int w, int h,
                                               int gx0, int gy0, StepConst C, int nlv, int lts) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)w * h) return;
  const int x = x0 + (int)(e % w), y = y0 + (int)(e / w);
  const int gx = gx0 + x, gy = gy0 + y;
  double a = 0.0;
  if (gx >= 0 && gx < C.nx && gy >= 0 && gy < C.ny) {
    const int64_t ncol = pair_sep_ncol(C.E, C.nx);
    const double *sxp = C.lsx + (gx + 2 * C.E);
    const double *ty = C.lty + (int64_t)(gy + 2 * C.E) * lts;
    a = sxp[(int64_t)nlv * ncol] * ty[nlv];
    for (int l = 0; l < nlv; ++l) a = fma(sxp[(int64_t)l * ncol], ty[l], a);
  }
  out[(int64_t)y * pitch + x] = a;
}

// compute_l2 / compute_linf partials (:96-113)
__global__ __launch_bounds__(256) void k_norms(const double *u, int64_t pitch,
                                               int bx, int by, int gx0,
                                               int gy0, StepConst C,
                                               NormPartial *out) {
#pragma clang fp contract(off)
  // (u - w)^2 with w = (ct*sin x)*sin y rounded exactly as compute_l2 does
  double s = 0.0, m = 0.0;
  const int64_t n = (int64_t)bx * by;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * 256) {
    const int x = (int)(e % bx), y = (int)(e / bx);
    const double w = (C.ct * C.sxt[gx0 + x + C.E]) * C.syt[gy0 + y + C.E];
    const double d = u[(int64_t)y * pitch + x] - w;
    s += d * d;
    m = fmax(m, fabs(d));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off);
    m = fmax(m, __shfl_xor(m, off));
  }
  __shared__ double ss[4], sm[4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    ss[wv] = s;
    sm[wv] = m;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[blockIdx.x].l2 = (ss[0] + ss[1]) + (ss[2] + ss[3]);
    out[blockIdx.x].linf = fmax(fmax(sm[0], sm[1]), fmax(sm[2], sm[3]));
  }
}

// ----------------------------------------------------------------------------
// launchers

static int check_launch() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// Fast-kernel variants, instantiated in nlh_fast_e*.hip (parallel build):
//   E = 1..16        128-column strips (R = 2); E <= 8 also 256-column (R = 4)
//                    and 64-column (R = 1)
// E = 17..48 run k_wide (nlh_wide.h); larger horizons run k_weighted (J = 1,
// to eps 52) or k_exact.
#define NLH_FAST_EXTERN(E, R)                                                            \
  extern template int launch_fast_er<E, R, true>(const RectList &, const StepConst &, hipStream_t); \
  extern template int launch_fast_er<E, R, false>(const RectList &, const StepConst &, hipStream_t);
NLH_FAST_EXTERN(1, 2) NLH_FAST_EXTERN(2, 2) NLH_FAST_EXTERN(3, 2) NLH_FAST_EXTERN(4, 2)
NLH_FAST_EXTERN(5, 2) NLH_FAST_EXTERN(6, 2) NLH_FAST_EXTERN(7, 2) NLH_FAST_EXTERN(8, 2)
NLH_FAST_EXTERN(9, 2) NLH_FAST_EXTERN(10, 2) NLH_FAST_EXTERN(11, 2) NLH_FAST_EXTERN(12, 2)
NLH_FAST_EXTERN(13, 2) NLH_FAST_EXTERN(14, 2) NLH_FAST_EXTERN(15, 2) NLH_FAST_EXTERN(16, 2)
NLH_FAST_EXTERN(1, 4) NLH_FAST_EXTERN(2, 4) NLH_FAST_EXTERN(3, 4) NLH_FAST_EXTERN(4, 4)
NLH_FAST_EXTERN(5, 4) NLH_FAST_EXTERN(6, 4) NLH_FAST_EXTERN(7, 4) NLH_FAST_EXTERN(8, 4)
NLH_FAST_EXTERN(1, 1) NLH_FAST_EXTERN(2, 1) NLH_FAST_EXTERN(3, 1) NLH_FAST_EXTERN(4, 1)
NLH_FAST_EXTERN(5, 1) NLH_FAST_EXTERN(6, 1) NLH_FAST_EXTERN(7, 1) NLH_FAST_EXTERN(8, 1)
NLH_FAST_EXTERN(9, 1) NLH_FAST_EXTERN(10, 1) NLH_FAST_EXTERN(11, 1) NLH_FAST_EXTERN(12, 1)
NLH_FAST_EXTERN(13, 1) NLH_FAST_EXTERN(14, 1) NLH_FAST_EXTERN(15, 1) NLH_FAST_EXTERN(16, 1)

// Large horizons (nlh_wide.h), instantiated in nlh_wide_e*.hip for E = 17..48
#define NLH_WIDE_EXTERN(E)                                                             \
  extern template int launch_wide_e<E, true>(const RectList &, const StepConst &, hipStream_t); \
  extern template int launch_wide_e<E, false>(const RectList &, const StepConst &, hipStream_t); \
  extern template int wide_blocks_per_cu_e<E>();
NLH_WIDE_EXTERN(17) NLH_WIDE_EXTERN(18) NLH_WIDE_EXTERN(19) NLH_WIDE_EXTERN(20)
NLH_WIDE_EXTERN(21) NLH_WIDE_EXTERN(22) NLH_WIDE_EXTERN(23) NLH_WIDE_EXTERN(24)
NLH_WIDE_EXTERN(25) NLH_WIDE_EXTERN(26) NLH_WIDE_EXTERN(27) NLH_WIDE_EXTERN(28)
NLH_WIDE_EXTERN(29) NLH_WIDE_EXTERN(30) NLH_WIDE_EXTERN(31) NLH_WIDE_EXTERN(32)
NLH_WIDE_EXTERN(33) NLH_WIDE_EXTERN(34) NLH_WIDE_EXTERN(35) NLH_WIDE_EXTERN(36)
NLH_WIDE_EXTERN(37) NLH_WIDE_EXTERN(38) NLH_WIDE_EXTERN(39) NLH_WIDE_EXTERN(40)
NLH_WIDE_EXTERN(41) NLH_WIDE_EXTERN(42) NLH_WIDE_EXTERN(43) NLH_WIDE_EXTERN(44)
NLH_WIDE_EXTERN(45) NLH_WIDE_EXTERN(46) NLH_WIDE_EXTERN(47) NLH_WIDE_EXTERN(48)
NLH_WIDE_EXTERN(49) NLH_WIDE_EXTERN(50) NLH_WIDE_EXTERN(51) NLH_WIDE_EXTERN(52)
NLH_WIDE_EXTERN(53) NLH_WIDE_EXTERN(54) NLH_WIDE_EXTERN(55) NLH_WIDE_EXTERN(56)
NLH_WIDE_EXTERN(57) NLH_WIDE_EXTERN(58) NLH_WIDE_EXTERN(59) NLH_WIDE_EXTERN(60)
NLH_WIDE_EXTERN(61) NLH_WIDE_EXTERN(62) NLH_WIDE_EXTERN(63) NLH_WIDE_EXTERN(64)

// k_wide: compile-time instances for eps 17..64 (nlh_wide.h)
bool wide_supported(int E) { return E >= 17 && E <= 64; }

#define NLH_WIDE_CASES(X)                                                                          \
  X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32) \
  X(33) X(34) X(35) X(36) X(37) X(38) X(39) X(40) X(41) X(42) X(43) X(44) X(45) X(46) X(47) X(48) \
  X(49) X(50) X(51) X(52) X(53) X(54) X(55) X(56) X(57) X(58) X(59) X(60) X(61) X(62) X(63) X(64)

int wide_blocks_per_cu(int E) {
  switch (E) {
#define NLH_CASEWO(EE) \
  case EE:             \
    return wide_blocks_per_cu_e<EE>();
    NLH_WIDE_CASES(NLH_CASEWO)
#undef NLH_CASEWO
    default:
      return 0;
  }
}

int launch_wide(const RectList &rl, const StepConst &c, bool test, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (c.E) {
#define NLH_CASEW(EE) \
  case EE:            \
    return test ? launch_wide_e<EE, true>(rl, c, st) : launch_wide_e<EE, false>(rl, c, st);
    NLH_WIDE_CASES(NLH_CASEW)
#undef NLH_CASEW
    default:
      return -1;
  }
}

int pair_pad_rows() { return kPairPadRows; }

// Two-step pass (nlh_pair.h), instantiated in nlh_pair_e*.hip for E = 1..16
#define NLH_PAIR_EXTERN(E) \
  extern template int launch_pair_e<E>(const RectList &, const StepConst &, int, hipStream_t); \
  extern template int pair_blocks_per_cu_e<E>(int);
NLH_PAIR_EXTERN(1) NLH_PAIR_EXTERN(2) NLH_PAIR_EXTERN(3) NLH_PAIR_EXTERN(4)
NLH_PAIR_EXTERN(5) NLH_PAIR_EXTERN(6) NLH_PAIR_EXTERN(7) NLH_PAIR_EXTERN(8)
NLH_PAIR_EXTERN(9) NLH_PAIR_EXTERN(10) NLH_PAIR_EXTERN(11) NLH_PAIR_EXTERN(12)
NLH_PAIR_EXTERN(13) NLH_PAIR_EXTERN(14) NLH_PAIR_EXTERN(15) NLH_PAIR_EXTERN(16)

// E = 15 spills registers in k_pair_split under hipcc 7.2 (424 bytes of
// scratch per lane): the single-step k_fast is faster there
// (profiles/r01/pair_v4/tune_eps_split.jsonl).  E = 13 spilled too before
// row pairs; with them it fits (230 VGPRs, two waves per SIMD)
bool pair_supported(int E) { return (E >= 1 && E <= 14) || E == 16; }

int pair_strip_width(int E) { return 128 - 2 * E; }

int pair_blocks_per_cu(int E, int variant) {
  switch (E) {
#define NLH_CASEO(EE) \
  case EE:            \
    return pair_blocks_per_cu_e<EE>(variant);
    NLH_CASEO(1) NLH_CASEO(2) NLH_CASEO(3) NLH_CASEO(4) NLH_CASEO(5) NLH_CASEO(6)
    NLH_CASEO(7) NLH_CASEO(8) NLH_CASEO(9) NLH_CASEO(10) NLH_CASEO(11) NLH_CASEO(12)
    NLH_CASEO(13) NLH_CASEO(14) NLH_CASEO(15) NLH_CASEO(16)
#undef NLH_CASEO
    default:
      return 0;
  }
}

int launch_pair(const RectList &rl, const StepConst &c, int variant, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (c.E) {
#define NLH_CASEP(EE) \
  case EE:            \
    return launch_pair_e<EE>(rl, c, variant, st);
    NLH_CASEP(1) NLH_CASEP(2) NLH_CASEP(3) NLH_CASEP(4) NLH_CASEP(5) NLH_CASEP(6)
    NLH_CASEP(7) NLH_CASEP(8) NLH_CASEP(9) NLH_CASEP(10) NLH_CASEP(11) NLH_CASEP(12)
    NLH_CASEP(13) NLH_CASEP(14) NLH_CASEP(15) NLH_CASEP(16)
#undef NLH_CASEP
    default:
      return -1;
  }
}

bool fast_supported(int E) { return E >= 1 && E <= 64; }

int fast_lanes_cols(int E, int want_r) {
  if (E > 16 || want_r == 1) return 1;
  return (want_r == 4 && E <= 8) ? 4 : 2;
}

int fast_strip_width(int E, int r) { return 64 * fast_lanes_cols(E, r); }

int fast_seg_min(int E) { return 2 * E; }

int launch_fast(const RectList &rl, const StepConst &c, bool test, int want_r, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  const int r = fast_lanes_cols(c.E, want_r);
#define NLH_CASE(EE, RR)                                                                \
  if (c.E == EE && r == RR)                                                            \
    return test ? launch_fast_er<EE, RR, true>(rl, c, st) : launch_fast_er<EE, RR, false>(rl, c, st);
  NLH_CASE(1, 2) NLH_CASE(2, 2) NLH_CASE(3, 2) NLH_CASE(4, 2) NLH_CASE(5, 2) NLH_CASE(6, 2)
  NLH_CASE(7, 2) NLH_CASE(8, 2) NLH_CASE(9, 2) NLH_CASE(10, 2) NLH_CASE(11, 2) NLH_CASE(12, 2)
  NLH_CASE(13, 2) NLH_CASE(14, 2) NLH_CASE(15, 2) NLH_CASE(16, 2)
  NLH_CASE(1, 4) NLH_CASE(2, 4) NLH_CASE(3, 4) NLH_CASE(4, 4) NLH_CASE(5, 4) NLH_CASE(6, 4)
  NLH_CASE(7, 4) NLH_CASE(8, 4)
  NLH_CASE(1, 1) NLH_CASE(2, 1) NLH_CASE(3, 1) NLH_CASE(4, 1) NLH_CASE(5, 1) NLH_CASE(6, 1)
  NLH_CASE(7, 1) NLH_CASE(8, 1) NLH_CASE(9, 1) NLH_CASE(10, 1) NLH_CASE(11, 1) NLH_CASE(12, 1)
  NLH_CASE(13, 1) NLH_CASE(14, 1) NLH_CASE(15, 1) NLH_CASE(16, 1)
#undef NLH_CASE
  return -1;
}

// k_exact_lds's tile(s) at two workgroups per CU at least
bool exact_lds_ok(int E, bool test) {
  return (size_t)(64 + 2 * E) * (16 + 2 * E) * sizeof(double) * (test ? 2 : 1) <= 80 * 1024;
}

int launch_exact(const RectList &rl, const StepConst &c, bool test, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool wt = c.influence != 0;
  if (exact_lds_ok(c.E, test)) {  // rects built with 16-row segments (build_rectlists)
    const size_t shm = (size_t)(64 + 2 * c.E) * (16 + 2 * c.E) * sizeof(double) * (test ? 2 : 1);
    if (test && wt)
      hipLaunchKernelGGL((k_exact_lds<true, true>), dim3(rl.nwork), dim3(256), shm, st, rl, c);
    else if (test)
      hipLaunchKernelGGL((k_exact_lds<true, false>), dim3(rl.nwork), dim3(256), shm, st, rl, c);
    else if (wt)
      hipLaunchKernelGGL((k_exact_lds<false, true>), dim3(rl.nwork), dim3(256), shm, st, rl, c);
    else
      hipLaunchKernelGGL((k_exact_lds<false, false>), dim3(rl.nwork), dim3(256), shm, st, rl, c);
    return check_launch();
  }
  if (test && wt)
    hipLaunchKernelGGL((k_exact<true, false, true>), dim3(rl.nwork), dim3(256), 0, st, rl, c);
  else if (test)
    hipLaunchKernelGGL((k_exact<true, false, false>), dim3(rl.nwork), dim3(256), 0, st, rl, c);
  else if (wt)
    hipLaunchKernelGGL((k_exact<false, false, true>), dim3(rl.nwork), dim3(256), 0, st, rl, c);
  else
    hipLaunchKernelGGL((k_exact<false, false, false>), dim3(rl.nwork), dim3(256), 0, st, rl, c);
  return check_launch();
}

int launch_exact_sum(const RectList &rl, const StepConst &c, void *stream) {
  if (c.influence != 0)
    hipLaunchKernelGGL((k_exact<false, true, true>), dim3(rl.nwork), dim3(256), 0,
                       (hipStream_t)stream, rl, c);
  else
    hipLaunchKernelGGL((k_exact<false, true, false>), dim3(rl.nwork), dim3(256), 0,
                       (hipStream_t)stream, rl, c);
  return check_launch();
}

// the (64+2E) x (16+2E) fp64 tile within the 160 KB LDS of a CU: E <= 52
bool weighted_supported(int E) {
  return E >= 1 && (size_t)(64 + 2 * E) * (16 + 2 * E) * sizeof(double) <= 160 * 1024;
}

int launch_weighted(const RectList &rl, const StepConst &c, bool test, void *stream) {
  const size_t shm = (size_t)(64 + 2 * c.E) * (16 + 2 * c.E) * sizeof(double);
  const size_t shm_col = shm + (size_t)(c.E + 1) * (c.E + 1) * sizeof(double);
  if (shm_col <= 160 * 1024) {  // the column kernel with J in LDS (eps <= 48)
    if (test)
      hipLaunchKernelGGL((k_weighted_col<true>), dim3(rl.nwork), dim3(256), shm_col, (hipStream_t)stream, rl, c);
    else
      hipLaunchKernelGGL((k_weighted_col<false>), dim3(rl.nwork), dim3(256), shm_col, (hipStream_t)stream, rl, c);
    return check_launch();
  }
  if (test)
    hipLaunchKernelGGL((k_weighted<true>), dim3(rl.nwork), dim3(256), shm, (hipStream_t)stream, rl, c);
  else
    hipLaunchKernelGGL((k_weighted<false>), dim3(rl.nwork), dim3(256), shm, (hipStream_t)stream, rl, c);
  return check_launch();
}

int launch_copies(const CopyList &cl, void *stream) {
  if (cl.nwork <= 0) return 0;
  hipLaunchKernelGGL(k_copies, dim3(cl.nwork), dim3(256), 0, (hipStream_t)stream, cl);
  return check_launch();
}

int launch_init_test(double *u, int64_t pitch, int32_t bx, int32_t by,
                     int32_t gx0, int32_t gy0, const StepConst &c, void *stream) {
  const int64_t n = (int64_t)bx * by;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_init_test, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, u, pitch, bx, by, gx0, gy0, c);
  return check_launch();
}

int launch_fill_w0(double *u, int64_t pitch, int32_t xl, int32_t bx, int32_t by, int32_t halo,
                   int32_t gx0, int32_t gy0, const StepConst &c, void *stream) {
  (void)bx;
  const int rows = by + 2 * halo;
  const int64_t n = pitch * rows;
  hipLaunchKernelGGL(k_fill_w0, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, u, pitch, xl, rows, halo, gx0, gy0, c);
  return check_launch();
}

int launch_lw_sep(double *out, int64_t pitch, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t gx0,
                  int32_t gy0, const StepConst &c, int32_t nlv, int32_t lts, void *stream) {
  const int64_t n = (int64_t)w * h;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_lw_sep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, out, pitch,
                     x0, y0, w, h, gx0, gy0, c, nlv, lts);
  return check_launch();
}

// an empty launch: the fixed cost of one launch between two timing events,
// subtracted from the busy time of each stencil launch (nlh_kernel_timing 2)
__global__ __launch_bounds__(64) void k_noop() {}

int launch_noop(void *stream) {
  hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, (hipStream_t)stream);
  return check_launch();
}

int norm_workgroups(int32_t bx, int32_t by) {
  const int64_t n = (int64_t)bx * by;
  int64_t g = (n + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

int launch_norms(const double *u, int64_t pitch, int32_t bx, int32_t by,
                 int32_t gx0, int32_t gy0, const StepConst &c, NormPartial *out,
                 void *stream) {
  hipLaunchKernelGGL(k_norms, dim3(norm_workgroups(bx, by)), dim3(256), 0,
                     (hipStream_t)stream, u, pitch, bx, by, gx0, gy0, c, out);
  return check_launch();
}

}  // namespace nlh