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

#include "nlh_device.h"

namespace nlh {

// ----------------------------------------------------------------------------
// helpers

// XCD-aware bijective remap: hardware deals workgroup ids round-robin over
// the 8 XCDs; give each XCD a contiguous range of work items so that strips
// sharing halo columns / warm-up rows hit the same L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7, l = bid >> 3;
  return (x < r) ? x * (q + 1) + l : r * (q + 1) + (x - r) * q + l;
}

__device__ __forceinline__ int find_rect(const RectList &L, int work) {
  int ri = 0;
  for (int k = 1; k < L.nrects; ++k) ri = (work >= L.r[k].wg_begin) ? k : ri;
  return ri;
}

// floor(sqrt(E^2 - d^2)) == (long)sqrt((double)(E*E - d*d)) of the
// reference's len_1d_line (:231) for every integer argument < 2^52.
__host__ __device__ constexpr int clen(int E, int d) {
  int L = 0;
  while ((L + 1) * (L + 1) <= E * E - d * d) ++L;
  return L;
}

__host__ __device__ constexpr int pow2_ceil(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

__host__ __device__ constexpr int disk_count(int E) {
  int n = 0;
  for (int d = -E; d <= E; ++d) n += 2 * clen(E, d < 0 ? -d : d) + 1;
  return n;
}

// One 16-byte-per-lane LDS-DMA: LDS[lds + 16*lane] <- global[g].
__device__ __forceinline__ void dma16(const void *g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(g), "s"(lds)
               : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(N) : "memory");
}

// NCH 16-byte chunks starting at g -> LDS starting at lds.
template <int NCH>
__device__ __forceinline__ void dma_chunks(const double *g, uint32_t lds,
                                           int lane) {
#pragma unroll
  for (int k = 0; k < (NCH + 63) / 64; ++k) {
    const double *src = g + 2 * (k * 64 + lane);
    if (k * 64 + 64 <= NCH) {
      dma16(src, lds + k * 1024);
    } else if (lane < NCH - k * 64) {
      dma16(src, lds + k * 1024);
    }
  }
}

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// ----------------------------------------------------------------------------
// k_exact: bit-parity kernel.  64x4 nodes per 256-thread workgroup.
template <bool TEST, bool SUMONLY>
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
  // sum_local (:256-270): sx outer, sy inner; out-of-domain halo cells are 0
  for (int dx = -E; dx <= E; ++dx) {
    const int len = C.lens[dx < 0 ? -dx : dx];
    const double *col = u + dx;
    for (int dy = -len; dy <= len; ++dy)
      res += ((C.c2d * (col[(int64_t)dy * p] - ui)) * C.dh2);
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
    for (int dx = -E; dx <= E; ++dx) {
      const int len = C.lens[dx < 0 ? -dx : dx];
      const int sx = gx + dx;
      const bool inx = (sx >= 0) && (sx < C.nx);
      const double cx = C.ct * C.sxt[sx + E];
      for (int dy = -len; dy <= len; ++dy) {
        const int sy = gy + dy;
        const bool in = inx && (sy >= 0) && (sy < C.ny);
        const double wv = in ? (cx * C.syt[sy + E]) : 0.0;
        r2 -= ((C.c2d * (wv - wpos)) * C.dh2);
      }
    }
    out += r2 * C.dt;
  }
  R.un[(int64_t)y * p + x] = out;
}

// ----------------------------------------------------------------------------
// k_fast: nested-window strip sweep.  See the file header.
//   E  horizon, R columns per lane (strip = 64*R columns), D rows in flight.
//
// Per wave: one strip of W = 64*R output columns over one segment of rows.
// Input rows stream through an LDS ring of K = next_pow2(E+D+1) slots
// (LDS-DMA issued D rows ahead); a row stays in the ring E rows after its
// window was consumed, so the centre value u(x, y) of the update is read back
// from it (slot arithmetic is a mask, no register shifting).  Odd segments sweep upwards
// so that the 2E rows two neighbouring segments both read are fetched at the
// same time (L2 hits instead of a second trip to HBM); work items run
// strip-fastest so horizontally adjacent strips, which share EP halo
// columns, are co-resident on one XCD.
template <int E, int R, int D, bool TEST>
__global__ __launch_bounds__(64) void k_fast(RectList L, StepConst C) {
  constexpr int P = 2 * E + 1;          // accumulator period (static unroll)
  constexpr int W = 64 * R;             // strip width (outputs)
  constexpr int EP = (E + 1) & ~1;      // halo columns staged per side
  constexpr int RW = W + 2 * EP;        // doubles per ring row
  constexpr int NCH = RW / 2;           // 16-byte chunks per row
  constexpr int K = pow2_ceil(E + D + 1);  // ring slots (power of two)
  constexpr int GU = (NCH + 63) / 64;   // DMA instructions per u row
  constexpr int GL = TEST ? (W / 2 + 63) / 64 : 0;  // per L_h[W0] row
  constexpr int G = GU + GL;
  constexpr int OFF = EP - E;           // window start inside a staged row
  static_assert(D >= 1, "prefetch distance");
  static_assert(D * G < 64, "vmcnt range");

  __shared__ __attribute__((aligned(16))) double ring[K * RW + (TEST ? K * W : 0)];
  double *lwr = ring + K * RW;  // L_h[W0] ring (TEST)

  const int lane = (int)threadIdx.x;
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &Rc = L.r[ri];
  const int local = work - Rc.wg_begin;
  const int strip = local % Rc.nstrip, seg = local / Rc.nstrip;
  const int x0 = Rc.x0 + strip * W;
  const int Y0 = Rc.y0 + seg * C.seg_h;
  const int Y1 = min(Y0 + C.seg_h, Rc.y1);
  const int n_in = (Y1 - Y0) + 2 * E;   // input rows Y0-E .. Y1+E-1
  const bool up = (seg & 1) != 0;       // sweep direction
  const int64_t pitch = Rc.pitch;
  const int64_t stride = up ? -pitch : pitch;
  const int yfirst = up ? (Y1 + E - 1) : (Y0 - E);  // block-local row of input 0

  const double *g0 = Rc.u + (int64_t)yfirst * pitch + (x0 - EP);
  // L_h[W0] row of the output emitted at iteration j (j >= 2E): Y0 + j - 2E
  // sweeping down, Y1 - 1 - (j - 2E) sweeping up
  const double *l0 = TEST ? Rc.lw + (int64_t)(up ? Y1 - 1 : Y0) * pitch + x0 : nullptr;
  const uint32_t lring = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  const uint32_t llw = __builtin_amdgcn_readfirstlane(lds_addr(lwr));

  const int xl = x0 + R * lane;  // first column of this lane
  double sxv[R];
  if (TEST) {
#pragma unroll
    for (int c = 0; c < R; ++c) {
      const int xc = min(xl + c, Rc.x1 - 1);
      sxv[c] = C.sxt[Rc.gx0 + xc + E];
      asm volatile("" ::"v"(sxv[c]));  // wait for it before the DMA stream
    }
  }

  // rows i of the u stream, and L_h rows for the output of iteration i
  auto issue = [&](int i, int slot) {
    const int rr = min(i, n_in - 1);
    dma_chunks<NCH>(g0 + (int64_t)rr * stride, lring + slot * RW * 8, lane);
    if (TEST) {
      const int lr = min(max(i - 2 * E, 0), n_in - 2 * E - 1);
      dma_chunks<W / 2>(l0 + (int64_t)lr * stride, llw + slot * W * 8, lane);
    }
  };

#pragma unroll
  for (int s = 0; s < D; ++s) issue(s, s);

  double acc[R][P];
#pragma unroll
  for (int c = 0; c < R; ++c)
#pragma unroll
    for (int j = 0; j < P; ++j) acc[c][j] = 0.0;
  int bs = 0;  // b % K
  for (int b = 0; b < n_in; b += P) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const int i = b + q;
      if (i < n_in) {
        const int slot = (bs + q) & (K - 1);
        issue(i + D, (bs + q + D) & (K - 1));
        wait_vmcnt<D * G>();

        // window of this lane: columns xl-E .. xl+R-1+E
        double w[R + 2 * E];
        const double *rowp = ring + slot * RW;
        if constexpr (R == 2) {
          constexpr int NB = (OFF + 2 * E + 2 + 1) / 2;
          const double2 *rp = reinterpret_cast<const double2 *>(rowp + 2 * lane);
          double buf[2 * NB];
#pragma unroll
          for (int k = 0; k < NB; ++k) {
            const double2 v = rp[k];
            buf[2 * k] = v.x;
            buf[2 * k + 1] = v.y;
          }
#pragma unroll
          for (int k = 0; k < R + 2 * E; ++k) w[k] = buf[OFF + k];
        } else {
#pragma unroll
          for (int k = 0; k < R + 2 * E; ++k) w[k] = rowp[OFF + lane + k];
        }

        // nested windows + scatter into the accumulators of rows i-d
#pragma unroll
        for (int c = 0; c < R; ++c) {
          double h = w[E + c];
#pragma unroll
          for (int Lv = 0; Lv <= E; ++Lv) {
            if (Lv > 0) h = h + (w[E + c - Lv] + w[E + c + Lv]);
#pragma unroll
            for (int d = -E; d <= E; ++d) {
              if (clen(E, d < 0 ? -d : d) == Lv) acc[c][(q + d + P) % P] += h;
            }
          }
        }

        // output of input row i-E is complete: accumulator (q - E) mod P
        const int so = (q + E + 1) % P;
        if (i >= 2 * E) {
          const int y = up ? (Y1 - 1 - (i - 2 * E)) : (Y0 + i - 2 * E);
          double out[R];
          const double *crow = ring + ((bs + q - E) & (K - 1)) * RW + EP + R * lane;
#pragma unroll
          for (int c = 0; c < R; ++c) {
            const double uc = crow[c];
            const double diff = fma(-C.nf, uc, acc[c][so]);
            out[c] = fma(diff, C.alpha, uc);
          }
          if (TEST) {
            const double syv = C.syt[Rc.gy0 + y + E];
            const double *lrow = lwr + slot * W + R * lane;
#pragma unroll
            for (int c = 0; c < R; ++c) {
              const double w0 = sxv[c] * syv;
              const double bsrc = -(C.st2pi * w0) - C.ct * lrow[c];
              out[c] = fma(bsrc, C.dt, out[c]);
            }
          }
          double *dst = Rc.un + (int64_t)y * pitch + xl;
          if constexpr (R == 2) {
            if (xl + 1 < Rc.x1) {
              *reinterpret_cast<double2 *>(dst) = make_double2(out[0], out[1]);
            } else if (xl < Rc.x1) {
              dst[0] = out[0];
            }
          } else {
            if (xl < Rc.x1) dst[0] = out[0];
          }
        }
#pragma unroll
        for (int c = 0; c < R; ++c) acc[c][so] = 0.0;
      }
    }
    bs = (bs + P) & (K - 1);
  }
  wait_vmcnt<0>();  // drain the clamped tail DMAs before the wave retires
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
                                                 int xl, int rows, int gx0,
                                                 int gy0, StepConst C) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= pitch * rows) return;
  const int px = (int)(e % pitch), py = (int)(e / pitch);
  const int gx = gx0 + px - xl, gy = gy0 + py - C.E;
  const bool in = gx >= 0 && gx < C.nx && gy >= 0 && gy < C.ny;
  u[e] = in ? C.sxt[gx + C.E] * C.syt[gy + C.E] : 0.0;
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

// compile-time dispatch table for the fast kernel: R = 2 (128-column strips)
// for every E <= 12, R = 4 (256-column strips) for E <= 8.
constexpr int kFastMaxE = 12;   // E >= 13 spills the accumulator file
constexpr int kFastMaxE4 = 8;   // widest E with a 256-column variant
constexpr int kFastD = 6;       // rows in flight per wave

template <int E, int R, bool TEST>
static int launch_fast_er(const RectList &rl, const StepConst &c, hipStream_t st) {
  hipLaunchKernelGGL((k_fast<E, R, kFastD, TEST>), dim3(rl.nwork), dim3(64), 0, st, rl, c);
  return check_launch();
}

template <int E>
static int launch_fast_dispatch(int e, int r, const RectList &rl, const StepConst &c, bool test,
                                hipStream_t st) {
  if constexpr (E == 0) {
    return -1;
  } else {
    if (e == E) {
      if constexpr (E <= kFastMaxE4) {
        if (r == 4)
          return test ? launch_fast_er<E, 4, true>(rl, c, st) : launch_fast_er<E, 4, false>(rl, c, st);
      }
      return test ? launch_fast_er<E, 2, true>(rl, c, st) : launch_fast_er<E, 2, false>(rl, c, st);
    }
    return launch_fast_dispatch<E - 1>(e, r, rl, c, test, st);
  }
}

bool fast_supported(int E) { return E >= 1 && (E <= kFastMaxE); }

int fast_lanes_cols(int E, int want_r) { return (want_r == 4 && E <= kFastMaxE4) ? 4 : 2; }

int fast_strip_width(int E, int r) { return 64 * fast_lanes_cols(E, r); }

int fast_seg_min(int E) { return 2 * E; }

int launch_fast(const RectList &rl, const StepConst &c, bool test, int r, void *stream) {
  if (!fast_supported(c.E)) return -1;
  return launch_fast_dispatch<kFastMaxE>(c.E, fast_lanes_cols(c.E, r), rl, c, test,
                                         (hipStream_t)stream);
}

int launch_exact(const RectList &rl, const StepConst &c, bool test, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (test)
    hipLaunchKernelGGL((k_exact<true, false>), dim3(rl.nwork), dim3(256), 0, st, rl, c);
  else
    hipLaunchKernelGGL((k_exact<false, false>), dim3(rl.nwork), dim3(256), 0, st, rl, c);
  return check_launch();
}

int launch_exact_sum(const RectList &rl, const StepConst &c, void *stream) {
  hipLaunchKernelGGL((k_exact<false, true>), dim3(rl.nwork), dim3(256), 0,
                     (hipStream_t)stream, rl, c);
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

int launch_fill_w0(double *u, int64_t pitch, int32_t xl, int32_t bx, int32_t by,
                   int32_t gx0, int32_t gy0, const StepConst &c, void *stream) {
  (void)bx;
  const int rows = by + 2 * c.E;
  const int64_t n = pitch * rows;
  hipLaunchKernelGGL(k_fill_w0, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, u, pitch, xl, rows, gx0, gy0, c);
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
