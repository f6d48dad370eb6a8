// nlh_prefix.h -- k_prefix_rt: single-step production / fast test-mode
// kernel for horizons past the compile-time k_wide instances (eps > 64), the
// horizon a run-time value.  Same operator as k_wide (reference sum_local,
// src/2d_nonlocal_serial.cpp:256-270 with J = 1; update :279-284; the
// reference accepts any --eps, :403):
//
//   S(x, y) = sum_{dy = -E..E} H_len(|dy|)(x, y + dy),
//   H_L(x, r) = sum_{|dx| <= L} u(x + dx, r) = P_r(x + L) - P_r(x - L - 1),
//
// P_r the prefix sum of input row r.  One wave per work item: 64 output
// columns (one per lane) x R output rows, accumulators in registers.  The
// wave streams the 2E + R input rows the block needs; per row each lane loads
// NV consecutive values of the staged window (64 + 2E <= 64 NV columns),
// sums them, scans the lane totals over the wave (DPP) and writes the
// prefix row to LDS; then every output row j of the block within the horizon
// adds H_len(|d|) = P(c + L) - P(c - L - 1), d = r - (y0 + j): two LDS reads,
// one subtraction, one add per (input row, output row) pair -- O(eps) per
// node instead of the O(eps^2) terms of k_exact.
//
// The per-offset prefix indices (c + L and c - L - 1 relative to the lane's
// centre, both 0 where |d| > E so the pair adds P(c) - P(c) = +0) come
// from a host table indexed by d + E + R, read with uniform (scalar) loads,
// so no pair branches.  Centre fold as k_wide: u' = alpha (S + (1/alpha - N)
// u), u read back from the field at the store; the fast test-mode source
// dt b enters as (dt/alpha) b with b = -(2 pi st) W0 - ct L_h[W0].
//
// The difference of two prefix sums of <= 64 NV values rounds at ~2^-44 of
// the row's magnitude; alpha ~ 1/N(eps) scales the disk sum of 2E + 1 of
// them, far inside the 1e-12 field-scale tolerance (tests/test_gpu_parity.py).
#pragma once

#include "nlh_device.h"
#include "nlh_kernel_common.h"
#include "nlh_rt.h"

namespace nlh {

// inclusive wave prefix sum (DPP row_shr 1/2/4/8, row_bcast 15/31), as k_wide
__device__ __forceinline__ double rt_wave_prefix(double x) {
  auto sh = [](double v, auto ctrl, auto rmask, auto bc) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), decltype(ctrl)::value,
                                               decltype(rmask)::value, 0xf, decltype(bc)::value);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), decltype(ctrl)::value,
                                               decltype(rmask)::value, 0xf, decltype(bc)::value);
    return __hiloint2double(hi, lo);
  };
  x += sh(x, std::integral_constant<int, 0x111>{}, std::integral_constant<int, 0xf>{}, std::true_type{});
  x += sh(x, std::integral_constant<int, 0x112>{}, std::integral_constant<int, 0xf>{}, std::true_type{});
  x += sh(x, std::integral_constant<int, 0x114>{}, std::integral_constant<int, 0xf>{}, std::true_type{});
  x += sh(x, std::integral_constant<int, 0x118>{}, std::integral_constant<int, 0xf>{}, std::true_type{});
  x += sh(x, std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xa>{}, std::false_type{});
  x += sh(x, std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xc>{}, std::false_type{});
  return x;
}

// NV staged values per lane (window of 64 NV columns: 64 + 2 E rounded up
// to even <= 64 NV), R output rows per work item (seg_rows of the rect
// list).  SKIP: input rows whose horizon misses some of the R output rows
// (the first and last R - 1 of the 2E + R) test each pair's row uniformly and
// skip it, instead of adding the table's zero offsets
//
// RUN: adjacent output rows j - 1, j whose row offsets d + 1, d have the same
// half-width (len changes slowly near |d| = 0: at eps 80, |d| <= 12 has two
// values) reuse the previous pair's H instead of two more LDS reads and a
// subtraction -- a uniform (scalar) test per pair
//
// CPL: output columns per lane (strips of 64 CPL columns); the lane's CPL
// prefix values at each offset are adjacent in LDS (one ds_read2_b64 for two
// columns), and the staged halo is shared by more columns
// PEEL: a full block's first and last R - 1 input rows add only the pairs of
// the outputs within their horizon (groups of 8 rows)
template <int NV, int R, bool TEST, bool SKIP = false, bool RUN = false, int CPL = 1, bool PEEL = false>
__global__ __launch_bounds__(64) void k_prefix_rt(RectList L, StepConst C, const int2 *__restrict__ tab) {
  constexpr int NPF = 64 * NV + 2;  // doubles per prefix slot: [0] = P(-1) = 0, [1 + k] = P(k)
  __shared__ __attribute__((aligned(16))) double pf[2][NPF];
  const int lane = (int)threadIdx.x;
  const int E = C.E;
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &Rc = L.r[ri];
  const int local = work - Rc.wg_begin;
  const int strip = local % Rc.nstrip, seg = local / Rc.nstrip;
  const int x0 = Rc.x0 + strip * (64 * CPL);
  const int y0 = Rc.y0 + seg * Rc.seg_rows;
  const int nout = min(R, Rc.y1 - y0);  // seg_rows == R (host)
  const int64_t pitch = Rc.pitch;
  const int xl = x0 + CPL * lane;  // the lane's first column
  if (lane == 0) {
    pf[0][0] = 0.0;
    pf[1][0] = 0.0;
  }
  // staged window: columns x0 - EP .. x0 - EP + 64 NV - 1 (EP = E rounded up
  // to even: 16-byte aligned rows, each lane's NV values two dwordx4 loads).
  // The columns past x0 + 63 + E feed no lane's window; they lie inside the
  // block's right padding (nlh_api.cpp sizes it for this window)
  const int EP = E + (E & 1);
  const double *gcol = Rc.u + (x0 - EP + NV * lane);
  auto load_row = [&](int r, double (&v)[NV]) __attribute__((always_inline)) {
    const double2 *g = reinterpret_cast<const double2 *>(gcol + (int64_t)r * pitch);
#pragma unroll
    for (int k = 0; k < NV / 2; ++k) {
      const double2 w = g[k];
      v[2 * k] = w.x;
      v[2 * k + 1] = w.y;
    }
  };
  double acc[R][CPL];
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc[j][c] = 0.0;

  const int rfirst = y0 - E, rend = y0 + nout + E;  // input rows [rfirst, rend)
  double cur[NV], nxt[NV];
  load_row(rfirst, cur);
  // one input row: its prefix row into LDS, then the pairs of outputs
  // JLO .. JHI (template constants; pairs past the horizon add +0)
  auto row = [&](int r, auto jlo_c, auto jhi_c) __attribute__((always_inline)) {
    constexpr int JLO = decltype(jlo_c)::value, JHI = decltype(jhi_c)::value;
    const int s = (r - rfirst) & 1;
    if (r + 1 < rend) load_row(r + 1, nxt);
    // prefix row of input row r into slot s
    double p[NV];
    p[0] = cur[0];
#pragma unroll
    for (int k = 1; k < NV; ++k) p[k] = p[k - 1] + cur[k];
    const double incl = rt_wave_prefix(p[NV - 1]);
    const double ex = incl - p[NV - 1];
    double *dst = &pf[s][1 + NV * lane];
#pragma unroll
    for (int k = 0; k < NV; ++k) dst[k] = ex + p[k];
    asm volatile("" ::: "memory");  // LDS is in order per wave: the reads below see every lane's write
    // pairs: output j <- d = r - (y0 + j); table entry d + E + R
    const int2 *t = tab + (r - y0 + E + R);
    const double *cen = &pf[s][1 + EP + CPL * lane];  // the lane's P(c), c = EP + CPL lane
    const int jlo = r - y0 - E, jhi = r - y0 + E;  // outputs within this row's horizon
    if constexpr (RUN) {
      double h = 0.0;
      int2 prev = make_int2(1, 1);  // no table entry
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int2 o = t[-j];  // {L, -L - 1}, or {0, 0} past the horizon
        if (o.x != prev.x || o.y != prev.y) h = cen[o.x] - cen[o.y];  // a new half-width
        prev = o;
        acc[j][0] += h;  // (RUN: one column per lane)
      }
    } else if (!SKIP || (jlo <= 0 && jhi >= R - 1)) {
#pragma unroll
      for (int j = JLO; j <= JHI; ++j) {
        const int2 o = t[-j];  // {L, -L - 1}, or {0, 0} past the horizon
#pragma unroll
        for (int c = 0; c < CPL; ++c) acc[j][c] += cen[o.x + c] - cen[o.y + c];
      }
    } else {
#pragma unroll
      for (int j = 0; j < R; ++j) {
        if (j >= jlo && j <= jhi) {
          const int2 o = t[-j];
#pragma unroll
          for (int c = 0; c < CPL; ++c) acc[j][c] += cen[o.x + c] - cen[o.y + c];
        }
      }
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int k = 0; k < NV; ++k) cur[k] = nxt[k];
  };
  using JAll0 = std::integral_constant<int, 0>;
  using JAllR = std::integral_constant<int, R - 1>;
  if (PEEL && nout == R && !RUN && !SKIP) {
    // a full block: input row t = r - y0 reaches outputs
    // max(0, t-E) .. min(R-1, t+E); its first R-1 rows (t < R-1-E) and last
    // R-1 rows (t > E) reach only part of the block.  Those rows run in groups
    // of PG whose pair ranges are the group's union (template constants), so
    // the pairs past the horizon -- (R-1)/(2E+R) of all, 14% at eps 96 --
    // shrink to the groups' rounding
    constexpr int PG = 8, NG = (R - 1 + PG - 1) / PG;
    int r = rfirst;
    static_for<NG>([&](auto gc) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
      constexpr int hi = PG * g + PG - 1 < R - 1 ? PG * g + PG - 1 : R - 2;  // t + E of the group's last row
#pragma unroll 1
      for (int k = PG * g; k <= hi; ++k, ++r) row(r, JAll0{}, std::integral_constant<int, hi>{});
    });
#pragma unroll 1
    for (; r <= y0 + E; ++r) row(r, JAll0{}, JAllR{});  // t in [R-1-E, E]: every output
    static_for<NG>([&](auto gc) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
      constexpr int lo = PG * g + 1;  // t - E of the group's first row
      constexpr int hi = PG * g + PG - 1 < R - 2 ? PG * g + PG - 1 : R - 2;
#pragma unroll 1
      for (int k = PG * g; k <= hi; ++k, ++r) row(r, std::integral_constant<int, lo>{}, JAllR{});
    });
  } else {
#pragma unroll 1
    for (int r = rfirst; r < rend; ++r) row(r, JAll0{}, JAllR{});
  }
  // u' = alpha (S + kc u) [+ (dt/alpha) b]: u(x, y) from the field
  static_assert(!RUN || CPL == 1, "RUN: one column per lane");
  const double alpha = C.alpha, kc = C.kc;
  const double qs = TEST ? C.dt / alpha : 0.0;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int x = xl + c;
    const bool emit = x < Rc.x1;
    const double sxv = TEST ? C.sxt[Rc.gx0 + min(x, Rc.x1 - 1) + E] : 0.0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (j < nout && emit) {
        const int64_t off = (int64_t)(y0 + j) * pitch + x;
        double a = fma(kc, Rc.u[off], acc[j][c]);
        if constexpr (TEST) {
          const double syv = C.syt[Rc.gy0 + y0 + j + E];
          const double b = -(C.st2pi * (sxv * syv)) - C.ct * Rc.lw[off];
          a = fma(qs, b, a);
        }
        Rc.un[off] = alpha * a;
      }
    }
  }
}

// k_prefix_rtc: k_prefix_rt for horizons whose staged window 64 + 2E passes
// 512 columns (eps > 224; VERDICT r4: no horizon falls back to k_exact).  The
// window is staged in nchk chunks of 64 NV columns: each chunk is loaded
// (the next chunk's loads in flight while this one scans), scanned over the
// wave and written to LDS on top of the running total of the chunks before
// it, so one LDS slot holds the prefix row of the whole window (dynamic LDS,
// 2 (64 NV nchk + 1) doubles).  The pair loop is k_prefix_rt's.  Prefix
// sums of up to 64 NV nchk values round at ~1e-13 of the row's magnitude;
// alpha ~ 1/N(eps) (N ~ pi eps^2) scales them far below the 1e-12 field-scale
// tolerance (tests/test_gpu_parity.py, eps 230 / 300).
template <int NV, int R, bool TEST>
__global__ __launch_bounds__(64) void k_prefix_rtc(RectList L, StepConst C, const int2 *__restrict__ tab,
                                                   int nchk) {
  extern __shared__ __attribute__((aligned(16))) double pfd[];
  const int npf = 64 * NV * nchk + 2;  // doubles per slot: [0] = P(-1) = 0, [1 + k] = P(k)
  const int lane = (int)threadIdx.x;
  const int E = C.E;
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &Rc = L.r[ri];
  const int local = work - Rc.wg_begin;
  const int strip = local % Rc.nstrip, seg = local / Rc.nstrip;
  const int x0 = Rc.x0 + strip * 64;
  const int y0 = Rc.y0 + seg * Rc.seg_rows;
  const int nout = min(R, Rc.y1 - y0);
  const int64_t pitch = Rc.pitch;
  const int xl = x0 + lane;
  if (lane == 0) {
    pfd[0] = 0.0;
    pfd[npf] = 0.0;
  }
  const int EP = E + (E & 1);
  const double *gcol = Rc.u + (x0 - EP + NV * lane);
  auto load_chunk = [&](int r, int c, double (&v)[NV]) __attribute__((always_inline)) {
    const double2 *g = reinterpret_cast<const double2 *>(gcol + (int64_t)r * pitch + 64 * NV * c);
#pragma unroll
    for (int k = 0; k < NV / 2; ++k) {
      const double2 w = g[k];
      v[2 * k] = w.x;
      v[2 * k + 1] = w.y;
    }
  };
  double acc[R];
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = 0.0;

  const int rfirst = y0 - E, rend = y0 + nout + E;
  double cur[NV], nxt[NV];
  load_chunk(rfirst, 0, cur);
  for (int r = rfirst; r < rend; ++r) {
    const int s = (r - rfirst) & 1;
    double *slot = pfd + s * npf;
    double carry = 0.0;
    for (int c = 0; c < nchk; ++c) {
      // the next chunk of this row, or the first chunk of the next row
      if (c + 1 < nchk)
        load_chunk(r, c + 1, nxt);
      else if (r + 1 < rend)
        load_chunk(r + 1, 0, nxt);
      double p[NV];
      p[0] = cur[0];
#pragma unroll
      for (int k = 1; k < NV; ++k) p[k] = p[k - 1] + cur[k];
      const double incl = rt_wave_prefix(p[NV - 1]);
      const double ex = carry + (incl - p[NV - 1]);
      double *dst = slot + 1 + 64 * NV * c + NV * lane;
#pragma unroll
      for (int k = 0; k < NV; ++k) dst[k] = ex + p[k];
      // the chunk's total (lane 63's inclusive sum) carries into the next
      carry += __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(incl), 63),
                                __builtin_amdgcn_readlane(__double2loint(incl), 63));
#pragma unroll
      for (int k = 0; k < NV; ++k) cur[k] = nxt[k];
    }
    asm volatile("" ::: "memory");  // LDS is in order per wave: the reads below see every lane's write
    const int2 *t = tab + (r - y0 + E + R);
    const double *cen = slot + 1 + EP + lane;  // the lane's P(c), c = EP + lane
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int2 o = t[-j];  // {L, -L - 1}, or {0, 0} past the horizon
      acc[j] += cen[o.x] - cen[o.y];
    }
    asm volatile("" ::: "memory");
  }
  const double alpha = C.alpha, kc = C.kc;
  const double qs = TEST ? C.dt / alpha : 0.0;
  const bool emit = xl < Rc.x1;
  const double sxv = TEST ? C.sxt[Rc.gx0 + min(xl, Rc.x1 - 1) + E] : 0.0;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (j < nout && emit) {
      const int64_t off = (int64_t)(y0 + j) * pitch + xl;
      double a = fma(kc, Rc.u[off], acc[j]);
      if constexpr (TEST) {
        const double syv = C.syt[Rc.gy0 + y0 + j + E];
        const double b = -(C.st2pi * (sxv * syv)) - C.ct * Rc.lw[off];
        a = fma(qs, b, a);
      }
      Rc.un[off] = alpha * a;
    }
  }
}

// k_prefix_rtw: k_prefix_rtc with W waves per workgroup sharing one staged
// prefix row (round 6).  The workgroup owns 64 W adjacent output columns x R
// rows; its window 64 W + 2E is staged in nchk chunks of 512 columns, chunk k
// scanned by wave k mod W, so each wave scans ~nchk / W chunks per row instead
// of the whole 64 + 2E window of its own 64 columns.  Per row:
//   scan:  each wave's chunks -> local prefix (no carry) into slot s, chunk
//          totals into tot[s];                                   s_barrier
//   carry: each wave adds the sum of the earlier chunks' totals to its
//          chunks' values (read-modify-write of its own LDS);    s_barrier
//   pairs: each wave's 64 columns, k_prefix_rt's pair loop on slot s.
// Slot s alternates per row, so the next row's scan (slot s ^ 1) never waits
// for the other waves' pair loops: two barriers per row.  Same prefix
// values as k_prefix_rtc up to the order of the carry additions (the carry
// is the sum of chunk totals, then added to the chunk's local prefix).
template <int NV, int R, bool TEST, int W>
__global__ __launch_bounds__(64 * W) void k_prefix_rtw(RectList L, StepConst C, const int2 *__restrict__ tab,
                                                       int nchk) {
  extern __shared__ __attribute__((aligned(16))) double pfd[];
  constexpr int CW = 64 * NV;          // columns per chunk
  const int npf = CW * nchk + 2;       // doubles per slot: [0] = P(-1) = 0, [1 + k] = P(k)
  double *tot = pfd + 2 * npf;         // [2][nchk] chunk totals
  const int lane = (int)threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int E = C.E;
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &Rc = L.r[ri];
  const int local = work - Rc.wg_begin;
  const int strip = local % Rc.nstrip, seg = local / Rc.nstrip;
  const int x0 = Rc.x0 + strip * (64 * W);
  const int y0 = Rc.y0 + seg * Rc.seg_rows;
  const int nout = min(R, Rc.y1 - y0);
  const int64_t pitch = Rc.pitch;
  const int xl = x0 + 64 * wv + lane;
  if (threadIdx.x == 0) {
    pfd[0] = 0.0;
    pfd[npf] = 0.0;
  }
  const int EP = E + (E & 1);
  const double *gcol = Rc.u + (x0 - EP + NV * lane);
  auto load_chunk = [&](int r, int c, double (&v)[NV]) __attribute__((always_inline)) {
    const double2 *g = reinterpret_cast<const double2 *>(gcol + (int64_t)r * pitch + CW * c);
#pragma unroll
    for (int k = 0; k < NV / 2; ++k) {
      const double2 w = g[k];
      v[2 * k] = w.x;
      v[2 * k + 1] = w.y;
    }
  };
  double acc[R];
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = 0.0;

  const int rfirst = y0 - E, rend = y0 + nout + E;
  // this wave's chunks: wv, wv + W, ..; the first one's values prefetched
  double cur[NV], nxt[NV];
  if (wv < nchk) load_chunk(rfirst, wv, cur);
  for (int r = rfirst; r < rend; ++r) {
    const int s = (r - rfirst) & 1;
    double *slot = pfd + s * npf;
    double *ts = tot + s * nchk;
    for (int c = wv; c < nchk; c += W) {
      // the wave's next chunk of this row, or its first chunk of the next row
      if (c + W < nchk)
        load_chunk(r, c + W, nxt);
      else if (r + 1 < rend)
        load_chunk(r + 1, wv, nxt);
      double p[NV];
      p[0] = cur[0];
#pragma unroll
      for (int k = 1; k < NV; ++k) p[k] = p[k - 1] + cur[k];
      const double incl = rt_wave_prefix(p[NV - 1]);
      const double ex = incl - p[NV - 1];
      double *dst = slot + 1 + CW * c + NV * lane;
#pragma unroll
      for (int k = 0; k < NV; ++k) dst[k] = ex + p[k];
      if (lane == 63) ts[c] = incl;
#pragma unroll
      for (int k = 0; k < NV; ++k) cur[k] = nxt[k];
    }
    __syncthreads();
    // carry: chunk c's values += total of chunks 0 .. c-1 (lane k holds the
    // inclusive sum of totals 0 .. k after a wave scan; nchk <= 64)
    {
      const double tk = lane < nchk ? ts[lane] : 0.0;
      const double ik = rt_wave_prefix(tk);
      for (int c = wv + (wv == 0 ? W : 0); c < nchk; c += W) {
        const double carry = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(ik), c - 1),
                                              __builtin_amdgcn_readlane(__double2loint(ik), c - 1));
        double *dst = slot + 1 + CW * c + NV * lane;
#pragma unroll
        for (int k = 0; k < NV; ++k) dst[k] += carry;
      }
    }
    __syncthreads();
    const int2 *t = tab + (r - y0 + E + R);
    const double *cen = slot + 1 + EP + 64 * wv + lane;  // the lane's P(c), c = EP + 64 wv + lane
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int2 o = t[-j];  // {L, -L - 1}, or {0, 0} past the horizon
      acc[j] += cen[o.x] - cen[o.y];
    }
  }
  const double alpha = C.alpha, kc = C.kc;
  const double qs = TEST ? C.dt / alpha : 0.0;
  const bool emit = xl < Rc.x1;
  const double sxv = TEST ? C.sxt[Rc.gx0 + min(xl, Rc.x1 - 1) + E] : 0.0;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (j < nout && emit) {
      const int64_t off = (int64_t)(y0 + j) * pitch + xl;
      double a = fma(kc, Rc.u[off], acc[j]);
      if constexpr (TEST) {
        const double syv = C.syt[Rc.gy0 + y0 + j + E];
        const double b = -(C.st2pi * (sxv * syv)) - C.ct * Rc.lw[off];
        a = fma(qs, b, a);
      }
      Rc.un[off] = alpha * a;
    }
  }
}

}  // namespace nlh
