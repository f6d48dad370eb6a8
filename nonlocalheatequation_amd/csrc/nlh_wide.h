// nlh_wide.h -- single-step production kernel for large horizons, k_wide
// (E = 17..48; C4's eps = 32 among them).  Same operator as k_fast (reference
// sum_local, src/2d_nonlocal_serial.cpp:256-270, J = 1; update :279-284), laid
// out for one wave per SIMD:
//
//   * one column per lane (64-column strips): the 2E+C live accumulators of a
//     column fill most of the 256 VGPRs a wave can address;
//   * accumulators in BLOCKS of C output rows: indexed by compile-time offsets
//     inside a chunk of C input rows and renamed (2E register moves) once per
//     chunk, so the row loop unrolls by C = 16 rows instead of k_fast's 2E+1.
//     At E = 32 k_fast's 65-row unroll is ~120 KB of code, about twice the
//     instruction cache; k_wide's chunk is a fraction of that;
//   * the window (2E+1 values per lane) streams from LDS in groups of levels,
//     the reads of group g+1 issued before the adds of group g, so it never
//     occupies more than a few registers;
//   * centre fold (u' = alpha (S + (1/alpha - N) u), as k_pair): no ring of
//     centre rows; the fast test-mode source dt*b(k) enters the accumulator of
//     output k at its centre row as (dt/alpha)*b(k).
//
// Input rows stream HBM -> LDS by LDS-DMA (global_load_lds_dwordx4) D rows
// ahead through a ring of K = pow2 >= D+1 slots, hand-counted vmcnt waits (as
// k_fast).  Every chunk processes C rows; rows past the segment re-read the
// last input row and only feed outputs that are never emitted.
//
// Indexing (sweep down; odd segments sweep up, mirrored): input row i = 0 ..
// n_in-1 is block row Y0-E+i, output row k = 0 .. seg-1 is block row Y0+k.
// Input i reaches outputs k = i-E-dy, dy in [-E, E], with the row window
// H_len(|dy|).  In chunk j (inputs i = C j + c) output k sits in accumulator
// a = k - (C j - 2E) = c + E - dy:  a = c + 2E is first touched (dy = -E,
// assigned), a = c + E takes the centre fold, a = c receives its last term.
// After the chunk a = 0 .. C-1 are complete (emitted), then a -> a - C.
#pragma once

#include "nlh_device.h"
#include "nlh_kernel_common.h"

namespace nlh {

constexpr int kWideC = 12;   // rows per chunk (unroll; profiles/r02/wide_bench_7.jsonl)
constexpr int kWideD = 6;    // input rows in flight
constexpr int kWideLG = 4;   // window levels per LDS read group

// number of row offsets dy in [-E, E] whose disk half-width len(|dy|) is L,
// and the t-th of them (ascending)
__host__ __device__ constexpr int wide_taps(int E, int L) {
  int n = 0;
  for (int dy = -E; dy <= E; ++dy)
    if (clen(E, dy < 0 ? -dy : dy) == L) ++n;
  return n;
}
__host__ __device__ constexpr int wide_tap_dy(int E, int L, int t) {
  for (int dy = -E; dy <= E; ++dy)
    if (clen(E, dy < 0 ? -dy : dy) == L && t-- == 0) return dy;
  return 0;
}

// Row pairs (RP): rows c (even, A) and c+1 (B) of a chunk reach output a at
// row offsets dy and dy+1.  Where len(|dy|) == len(|dy+1|) > 0 both add the
// same level: row A skips that tap and row B adds H_L(A) + H_L(B) once, one
// extra add per shared level (E = 32: 26 of the 128 taps of a row pair become
// 6 pair sums -- 20 adds fewer per row pair and column).
__host__ __device__ constexpr bool wide_shared(int E, int dy) {
  return dy >= -E && dy < E && clen(E, dy < 0 ? -dy : dy) > 0 &&
         clen(E, dy < 0 ? -dy : dy) == clen(E, dy + 1 < 0 ? -dy - 1 : dy + 1);
}
__host__ __device__ constexpr bool wide_level_shared(int E, int L) {
  for (int dy = -E; dy < E; ++dy)
    if (wide_shared(E, dy) && clen(E, dy < 0 ? -dy : dy) == L) return true;
  return false;
}

// the last level < L whose row window feeds some output (0: the centre column)
__host__ __device__ constexpr int wide_prev_used(int E, int L) {
  for (int l = L - 1; l > 0; --l)
    if (wide_taps(E, l) > 0) return l;
  return 0;
}

// p[LO] + .. + p[HI] as a balanced tree (depth log2 instead of HI-LO)
template <int LO, int HI, int N>
__device__ __forceinline__ double tree_sum(const double (&p)[N]) {
  if constexpr (LO == HI)
    return p[LO];
  else
    return tree_sum<LO, (LO + HI) / 2>(p) + tree_sum<(LO + HI) / 2 + 1, HI>(p);
}

// Inclusive prefix sum of x over the 64 lanes of the wave: Hillis-Steele
// within each 16-lane row (DPP row_shr 1, 2, 4, 8, zero-filled at the row
// start), then the row totals carried by row_bcast:15 / row_bcast:31.  fp64 as
// two 32-bit DPP moves per step.
__device__ __forceinline__ double wave_prefix_sum(double x) {
  auto sh = [](double v, auto ctrl, auto rmask, auto bc) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), decltype(ctrl)::value,
                                               decltype(rmask)::value, 0xf, decltype(bc)::value);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), decltype(ctrl)::value,
                                               decltype(rmask)::value, 0xf, decltype(bc)::value);
    return __hiloint2double(hi, lo);
  };
  using I = std::integral_constant<int, 0>;
  (void)sizeof(I);
  x += sh(x, std::integral_constant<int, 0x111>{}, std::integral_constant<int, 0xf>{}, std::true_type{});
  x += sh(x, std::integral_constant<int, 0x112>{}, std::integral_constant<int, 0xf>{}, std::true_type{});
  x += sh(x, std::integral_constant<int, 0x114>{}, std::integral_constant<int, 0xf>{}, std::true_type{});
  x += sh(x, std::integral_constant<int, 0x118>{}, std::integral_constant<int, 0xf>{}, std::true_type{});
  x += sh(x, std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xa>{}, std::false_type{});
  x += sh(x, std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xc>{}, std::false_type{});
  return x;
}

// ABL (diagnostics, timing only): 1 = a scheduling barrier between rows
// PS: row windows from a prefix sum of the staged row instead of the nested
// pair sums.  The lane's 16-byte chunk of the staged row (two, past 128
// doubles: E > 32) is summed, scanned over the wave (DPP; the second chunk
// adds the first scan's total) and written back as P(k) = staged[0] + .. +
// staged[k]; a used level L is then
// H_L = P(c+L) - P(c-L-1): two LDS reads and one subtraction per USED level
// (19 of 32 at E = 32, 24 of 40 at E = 40) instead of two reads and two adds
// per level.  The difference of two prefix sums of at most 160 values rounds at ~2^-45 of the
// row's magnitude: far inside the 1e-12 field-scale tolerance once alpha ~ 1/N
// scales the disk sum.
//
// PSPLIT (with PS): the two prefix reads of a level as separate ds_read_b64
// (2 LDS cycles each); left alone the compiler pairs them into one
// ds_read2_b64, which takes 8 (MI355X_MICROARCH.md LDS table)
//
// PA (with PS): prefix rows built PA rows ahead into a ring of PK prefix
// slots -- row i's 38 window reads hit a prefix row finished PA rows earlier,
// and the scan of row i+PA (its DPP chain and LDS write) is independent of
// row i's window sums, so the two interleave instead of serialising each row
// on scan -> LDS write -> LDS read.  Same arithmetic: bitwise equal to PA = 0.
//
// ILS (with PA, E <= 32): the scan reads and writes 64 full lanes of a padded
// prefix slot without exec-mask branches (lanes past the staged row read
// bytes no level ever uses) and without compiler barriers around it, so the
// row's window reads, the scan of row i + PA and the row's taps form one
// basic block and the scan's dependent DPP/add chain interleaves with the
// taps instead of running alone.  Same arithmetic: bitwise equal.
template <int E, int CH, bool TEST, int D = kWideD, int ABL = 0, int PIN = 1, bool AB = false, int OBP = 16,
          bool SPLIT8 = true, bool PS = false, int PA = 0, bool PSPLIT = false, bool ILS = false, bool NTS = false,
          bool RP = false, bool SP = false>
__global__ __launch_bounds__(64, 1) void k_wide(RectList L, StepConst C) {
  constexpr int W = 64;                 // output columns per strip
  constexpr int EP = (E + 1) & ~1;      // staged halo columns per side (16-B rows)
  constexpr int RW = W + 2 * EP;        // staged doubles per ring row
  constexpr int NCH = RW / 2;           // 16-byte chunks per row
  // AB: every row staged twice, copy B one column later than copy A and
  // OBP doubles further in LDS, shifting the banks the odd lanes read
  constexpr int RWS = AB ? 2 * RW + 2 * OBP : RW;  // doubles per ring slot
  constexpr int OB = RW + OBP;                     // copy B within a slot
  constexpr int K = pow2_ceil(D + 1);   // ring slots
  constexpr int GU = (AB ? 2 : 1) * ((NCH + 63) / 64);  // DMA instructions per u row
  constexpr int GL = TEST ? (W / 2 + 63) / 64 : 0;  // per L_h[W0] row
  constexpr int GS = TEST ? 1 : 0;  // the row's sin(2 pi y dh) pair (no scalar load per row)
  constexpr int G = GU + GL + GS;
  constexpr int NA = 2 * E + CH;        // live accumulators
  constexpr int NG = (E + kWideLG - 1) / kWideLG;  // level groups
  static_assert(D * G + CH < 64, "vmcnt range");
  static_assert(CH % PIN == 0, "rows per pin");
  static_assert(!RP || (CH % 2 == 0 && (PA > 0 || !PS)), "row pairs: even chunks; prefix-ahead rows or nested windows");

  static_assert(!PS || (RW <= 256 && !AB), "prefix-sum rows: at most four staged doubles per lane");
  static_assert(PA == 0 || (PS && PA < D), "prefix-ahead rows need prefix sums and landed rows");
  constexpr int PK = PA ? pow2_ceil(PA + 1) : 1;  // prefix-row slots
  static_assert(!ILS || (PA > 0 && RW <= 128), "interleaved scan: one 16-byte chunk per lane");
  constexpr int NPR = ILS ? 130 : RW + 2;          // doubles per prefix slot (16-B multiple)
  constexpr int NP = PS ? PK * NPR : 0;  // prefix row: pfx[1] = 0, pfx[2 + k] = P(k)
  __shared__ __attribute__((aligned(16))) double ring[K * RWS + (TEST ? K * W + 2 * K : 0) + NP];
  double *lwr = ring + K * RWS;  // L_h[W0] rows (TEST), same slots as the u rows
  double *syr = lwr + K * W;     // sin(2 pi y dh) pairs (TEST), same slots
  double *pfx = ring + K * RWS + (TEST ? K * W + 2 * K : 0);  // PS: prefix row

  const int lane = (int)threadIdx.x;
  if constexpr (PS) {
    if (lane < PK) pfx[lane * NPR + 1] = 0.0;  // P(-1) of every slot; the row writes start at [2]
  }
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &Rc = L.r[ri];
  const double *const ru = Rc.u;
  double *const run = Rc.un;
  const int rx1 = Rc.x1, rgx0 = Rc.gx0, rgy0 = Rc.gy0;
  const int local = work - Rc.wg_begin;
  const int nstrip = Rc.nstrip;
  const int strip = local % nstrip, seg = local / nstrip;
  const int x0 = Rc.x0 + strip * W;
  const int seg_h = Rc.seg_rows;
  const int Y0 = Rc.y0 + seg * seg_h;
  const int Y1 = min(Y0 + seg_h, Rc.y1);
  const int nout = Y1 - Y0;
  const int n_in = nout + 2 * E;
  const bool up = (seg & 1) != 0;
  const int64_t pitch = Rc.pitch;
  const int64_t stride = up ? -pitch : pitch;
  const int yfirst = up ? (Y1 + E - 1) : (Y0 - E);
  const double alpha = C.alpha, kc = C.kc;

  const int xl = x0 + lane;  // the column of this lane
  const bool emit = xl < rx1;
  double sxv = 0.0;
  if constexpr (TEST) sxv = C.sxt[rgx0 + min(xl, rx1 - 1) + E];

  // AB: window start of this lane, staged column (EP - E) + lane of copy A,
  // or of copy B one column earlier when that is odd
  const int s_l = EP - E + lane;
  const int lane_off = (s_l & 1) ? OB + s_l - 1 : s_l;
  const uint32_t lring = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  const uint32_t llw = __builtin_amdgcn_readfirstlane(lds_addr(lwr));
  const uint32_t lsy = __builtin_amdgcn_readfirstlane(lds_addr(syr));
  // table index of sin(2 pi y dh) for output k = i - E of input row i
  auto sy_index = [&](int i) {
    const int k = min(max(i - E, 0), nout - 1);
    return rgy0 + (up ? Y1 - 1 - k : Y0 + k) + E;
  };
  // u rows: running pointer clamped at the last input row
  const double *gnext = ru + (int64_t)yfirst * pitch + (x0 - EP);
  // L_h[W0] row of output k = i - E (the centre row of input i), fetched with
  // input row i into the same ring slot; rows -E .. nout+E-1 lie in the halo
  const double *l0 = TEST ? Rc.lw + (int64_t)(up ? Y1 - 1 : Y0) * pitch + x0 : nullptr;
  int fetched = 0;  // next input row to issue
  auto issue = [&]() __attribute__((always_inline)) {
    const int slot = fetched & (K - 1);
    if constexpr (TEST) {
      const int k = min(fetched, n_in - 1) - E;
      dma_chunks<W / 2>(l0 + (int64_t)k * stride, llw + slot * W * 8, lane);
      dma_chunks<1>(C.syt + (sy_index(fetched) & ~1), lsy + slot * 16, lane);
    }
    // default-policy (temporal) DMA: the neighbouring strips stage this row's
    // halo columns again through the same XCD's L2 (C4: 167-169 vs 164-166 G
    // node/s with nt, profiles/r04/first/wide_wpg.jsonl)
    dma_chunks<NCH, false, false>(gnext, lring + slot * RWS * 8, lane);
    if constexpr (AB) dma_chunks<NCH>(gnext + 1, lring + (slot * RWS + OB) * 8, lane);
    ++fetched;
    if (fetched < n_in) gnext += stride;
  };
#pragma unroll
  for (int s = 0; s < D; ++s) issue();

  // PS: prefix row of staged row r into prefix slot r mod PK
  auto scan_row = [&](int r) __attribute__((always_inline)) {
    const double *srow = ring + (r & (K - 1)) * RWS;
    double *dst = pfx + (r & (PK - 1)) * NPR + 2;
    if constexpr (ILS) {
      const double2 ab = *reinterpret_cast<const double2 *>(srow + 2 * lane);
      const double sv = wave_prefix_sum(ab.x + ab.y);
      *reinterpret_cast<double2 *>(dst + 2 * lane) = make_double2(sv - ab.y, sv);
      return;
    }
    double2 ab = make_double2(0.0, 0.0);
    if (2 * lane < RW) ab = *reinterpret_cast<const double2 *>(srow + 2 * lane);
    double2 cd = make_double2(0.0, 0.0);  // second chunk of the lane (E > 32)
    if constexpr (RW > 128)
      if (2 * (lane + 64) < RW) cd = *reinterpret_cast<const double2 *>(srow + 2 * (lane + 64));
    const double sv = wave_prefix_sum(ab.x + ab.y);
    double sw = 0.0;
    if constexpr (RW > 128) {
      const double tot = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(sv), 63),
                                          __builtin_amdgcn_readlane(__double2loint(sv), 63));
      sw = wave_prefix_sum(cd.x + cd.y) + tot;
    }
    asm volatile("" ::: "memory");
    if (2 * lane < RW) *reinterpret_cast<double2 *>(dst + 2 * lane) = make_double2(sv - ab.y, sv);
    if constexpr (RW > 128)
      if (2 * (lane + 64) < RW) *reinterpret_cast<double2 *>(dst + 2 * (lane + 64)) = make_double2(sw - cd.y, sw);
    asm volatile("" ::: "memory");  // in order per wave: later reads see every lane's write
  };
  if constexpr (PA > 0) {
    // prologue: prefix rows 0 .. PA-1 (row r landed: D-1-r rows may still fly)
    static_for<PA>([&](auto rc) __attribute__((always_inline)) {
      constexpr int r = decltype(rc)::value;
      wait_vmcnt<(D - 1 - r) * G>();
      scan_row(r);
    });
  }

  double acc[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) acc[a] = 0.0;
  double hsv[E + 1];  // RP: row A's windows at the shared levels, until row B

  const double qs = TEST ? C.dt / alpha : 0.0;
  const int nchunk = (n_in + CH - 1) / CH;
  bool full = false;  // the previous chunk stored CH output rows
  for (int j = 0; j < nchunk; ++j) {
    const int ibase = j * CH;
    auto row = [&](auto cc) __attribute__((always_inline)) {
      constexpr int c = decltype(cc)::value;
      if constexpr ((ABL & 1) != 0) __builtin_amdgcn_sched_barrier(0);
      const int i = ibase + c;
      issue();  // input row i + D
      // row i + PA landed.  Issued after its DMA: the DMAs of rows
      // i+PA+1 .. i+D, and for c + PA < D the CH output stores of the
      // previous chunk's end
      if constexpr (c + PA < D) {
        if (full)
          wait_vmcnt<(D - PA) * G + CH>();
        else
          wait_vmcnt<(D - PA) * G>();
      } else {
        wait_vmcnt<(D - PA) * G>();
      }
      // this lane's window: staged columns xl-E .. xl+E
      // this lane's window w[0 .. 2E] (w[E] its own column).  AB: read as
      // 16-byte pairs from copy A or B of the row, whichever has it aligned
      // (ds_read_b128: 4 LDS cycles per KB; 8-byte reads paired by the
      // compiler into ds_read2_b64 take 8, and LDS-bound the kernel)
      const double *wrow = AB ? ring + (i & (K - 1)) * RWS + lane_off
                              : ring + (i & (K - 1)) * RWS + (EP - E) + lane;
      auto wpair = [&](int k2) __attribute__((always_inline)) {  // w[2 k2], w[2 k2 + 1]
        return *reinterpret_cast<const double2 *>(wrow + 2 * k2);
      };
      double wl[NG][kWideLG], wr[NG][kWideLG];
      auto load_group = [&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value;
        constexpr int L0 = g * kWideLG + 1;
        constexpr int LN = L0 + kWideLG - 1 < E ? L0 + kWideLG - 1 : E;
        if constexpr (AB) {
          double lv[2 * kWideLG + 2], rv[2 * kWideLG + 2];
          constexpr int lk0 = (E - LN) / 2, lk1 = (E - L0) / 2;  // pairs covering w[E-LN .. E-L0]
          constexpr int rk0 = (E + L0) / 2, rk1 = (E + LN) / 2;  // pairs covering w[E+L0 .. E+LN]
#pragma unroll
          for (int k = lk0; k <= lk1; ++k) {
            const double2 v = wpair(k);
            lv[2 * (k - lk0)] = v.x;
            lv[2 * (k - lk0) + 1] = v.y;
          }
#pragma unroll
          for (int k = rk0; k <= rk1; ++k) {
            const double2 v = wpair(k);
            rv[2 * (k - rk0)] = v.x;
            rv[2 * (k - rk0) + 1] = v.y;
          }
#pragma unroll
          for (int t = 0; t < kWideLG; ++t) {
            if (L0 + t <= E) {
              wl[g][t] = lv[E - (L0 + t) - 2 * lk0];
              wr[g][t] = rv[E + (L0 + t) - 2 * rk0];
            }
          }
        } else if constexpr (SPLIT8) {
          // separate ds_read_b64 (2 LDS cycles per wave-instruction): a memory
          // barrier between the reads keeps the compiler from pairing them into
          // ds_read2_b64 (8 cycles for the same bytes); the kernel is LDS-bound
          // (SQ_LDS_IDX_ACTIVE 86% of cycles with the pairs, 548 vs 612 us per
          // step at 8192^2, eps 32 without them)
#pragma unroll
          for (int t = 0; t < kWideLG; ++t) {
            if (L0 + t <= E) {
              wl[g][t] = wrow[E - (L0 + t)];
              asm volatile("" ::: "memory");
              wr[g][t] = wrow[E + (L0 + t)];
              asm volatile("" ::: "memory");
            }
          }
        } else {
#pragma unroll
          for (int t = 0; t < kWideLG; ++t) {
            if (L0 + t <= E) {
              wl[g][t] = wrow[E - (L0 + t)];
              wr[g][t] = wrow[E + (L0 + t)];
            }
          }
        }
      };
      const double wc = AB ? ((E % 2 == 0) ? wpair(E / 2).x : wpair(E / 2).y) : wrow[E];
      if constexpr (PS && PA > 0) {
        // row i's prefix row was built PA rows ago: its window reads go out
        // first, the scan of row i + PA runs while they are in flight
        const double *pl = pfx + (i & (PK - 1)) * NPR + 2 + EP + lane;  // P(centre + k) at pl[k]
        double hp[E + 1], hm[E + 1];
        static_for<E>([&](auto lc) __attribute__((always_inline)) {
          constexpr int Lv = decltype(lc)::value + 1;
          if constexpr (wide_taps(E, Lv) > 0) {
            hp[Lv] = pl[Lv];
            if constexpr (PSPLIT) asm volatile("" ::: "memory");
            hm[Lv] = pl[-Lv - 1];
            if constexpr (PSPLIT) asm volatile("" ::: "memory");
          }
        });
        if constexpr (!ILS) asm volatile("" ::: "memory");  // the reads above are issued before the scan's write
        scan_row(i + PA);
        acc[c + 2 * E] = wc;
        acc[c] += wc;
        static_for<E>([&](auto lc) __attribute__((always_inline)) {
          constexpr int Lv = decltype(lc)::value + 1;
          if constexpr (wide_taps(E, Lv) > 0) {
            const double h = hp[Lv] - hm[Lv];
            constexpr bool sh = RP && wide_level_shared(E, Lv);
            double ps = h;
            if constexpr (sh && c % 2 == 0)
              hsv[Lv] = h;
            else if constexpr (sh)
              ps = hsv[Lv] + h;
            static_for<wide_taps(E, Lv)>([&](auto kk) __attribute__((always_inline)) {
              constexpr int dy = wide_tap_dy(E, Lv, decltype(kk)::value);
              if constexpr (RP && c % 2 == 0 && wide_shared(E, dy)) {
                // row B adds the pair sum
              } else if constexpr (RP && c % 2 == 1 && wide_shared(E, dy - 1)) {
                acc[c + E - dy] += ps;
              } else {
                acc[c + E - dy] += h;
              }
            });
          }
        });
      } else if constexpr (PS) {
        // prefix row of the staged row (slot i), then the used levels' windows
        const double *srow = ring + (i & (K - 1)) * RWS;
        double2 ab = make_double2(0.0, 0.0);
        if (2 * lane < RW) ab = *reinterpret_cast<const double2 *>(srow + 2 * lane);
        double2 cd = make_double2(0.0, 0.0);  // second chunk of the lane (E > 32)
        if constexpr (RW > 128)
          if (2 * (lane + 64) < RW) cd = *reinterpret_cast<const double2 *>(srow + 2 * (lane + 64));
        const double sv = wave_prefix_sum(ab.x + ab.y);
        double sw = 0.0;
        if constexpr (RW > 128) {
          const double tot = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(sv), 63),
                                              __builtin_amdgcn_readlane(__double2loint(sv), 63));
          sw = wave_prefix_sum(cd.x + cd.y) + tot;
        }
        asm volatile("" ::: "memory");
        if (2 * lane < RW) *reinterpret_cast<double2 *>(pfx + 2 + 2 * lane) = make_double2(sv - ab.y, sv);
        if constexpr (RW > 128)
          if (2 * (lane + 64) < RW)
            *reinterpret_cast<double2 *>(pfx + 2 + 2 * (lane + 64)) = make_double2(sw - cd.y, sw);
        asm volatile("" ::: "memory");  // in order per wave: the reads below see every lane's write
        acc[c + 2 * E] = wc;
        acc[c] += wc;
        const double *pl = pfx + 2 + EP + lane;  // P(centre column + k) at pl[k]
        auto plevel = [&](auto lc) __attribute__((always_inline)) {
          constexpr int Lv = decltype(lc)::value + 1;
          if constexpr (wide_taps(E, Lv) > 0) {
            const double ph = pl[Lv];
            if constexpr (PSPLIT) asm volatile("" ::: "memory");
            const double pm = pl[-Lv - 1];
            if constexpr (PSPLIT) asm volatile("" ::: "memory");
            const double h = ph - pm;
            auto tap = [&](auto kk) __attribute__((always_inline)) {
              constexpr int dy = wide_tap_dy(E, Lv, decltype(kk)::value);
              acc[c + E - dy] += h;
            };
            static_for<wide_taps(E, Lv)>(tap);
          }
        };
        static_for<E>(plevel);
      } else {
      load_group(std::integral_constant<int, 0>{});
      // dy = -E: first term of output a = c + 2E; dy = +E: last of a = c
      acc[c + 2 * E] = wc;
      acc[c] += wc;
      double core = wc;
      double pend = 0.0;  // p of levels not yet folded into core
      auto group = [&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value;
        // region = the next group's LDS reads + this group's adds: the
        // scheduler may not hoist later reads (register pressure) or sink
        // these adds past them
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (g + 1 < NG) load_group(std::integral_constant<int, g + 1>{});
        // the window sum grows by p_L = w[E-L] + w[E+L] per level; it is only
        // needed at levels some output uses, so the p of the levels between
        // two used ones are summed as a tree and folded in once (the same
        // adds as the level-by-level chain, a fraction of its depth).
        // Levels past the group's last used one carry over in `pend`.
        constexpr int L0 = g * kWideLG + 1;
        double pp[kWideLG];
#pragma unroll
        for (int t = 0; t < kWideLG; ++t)
          if (L0 + t <= E) pp[t] = wl[g][t] + wr[g][t];
        auto level = [&](auto tc) __attribute__((always_inline)) {
          constexpr int t = decltype(tc)::value;
          constexpr int Lv = L0 + t;
          if constexpr (Lv <= E && wide_taps(E, Lv) > 0) {
            constexpr int s0 = wide_prev_used(E, Lv) + 1;  // first level of this segment
            constexpr int lo = s0 > L0 ? s0 - L0 : 0;
            const double seg = tree_sum<lo, t>(pp);
            if constexpr (s0 < L0)  // the segment began in an earlier group
              core = core + (pend + seg);
            else
              core = core + seg;
            constexpr bool sh = RP && wide_level_shared(E, Lv);
            double ps = core;
            if constexpr (sh && c % 2 == 0)
              hsv[Lv] = core;
            else if constexpr (sh)
              ps = hsv[Lv] + core;
            auto tap = [&](auto kk) __attribute__((always_inline)) {
              constexpr int dy = wide_tap_dy(E, Lv, decltype(kk)::value);
              if constexpr (RP && c % 2 == 0 && wide_shared(E, dy)) {
                // row B adds the pair sum
              } else if constexpr (RP && c % 2 == 1 && wide_shared(E, dy - 1)) {
                acc[c + E - dy] += ps;
              } else {
                acc[c + E - dy] += core;
              }
            };
            static_for<wide_taps(E, Lv)>(tap);
          }
        };
        static_for<kWideLG>(level);
        // levels after the group's last used one: carried to the next group
        constexpr int LE = L0 + kWideLG - 1 < E ? L0 + kWideLG - 1 : E;
        constexpr int s0 = wide_prev_used(E, LE + 1) + 1;  // first unfolded level
        if constexpr (LE < E && s0 <= LE) {
          constexpr int lo = s0 > L0 ? s0 - L0 : 0;
          const double seg = tree_sum<lo, LE - L0>(pp);
          if constexpr (s0 < L0)
            pend = pend + seg;
          else
            pend = seg;
        }
      };
      static_for<NG>(group);
      }
      acc[c + E] = fma(kc, wc, acc[c + E]);
      if constexpr (TEST) {
        // b = -(2 pi st) W0 - ct L_h[W0] at output k = i - E
        const double syv = syr[2 * (i & (K - 1)) + (sy_index(i) & 1)];
        const double b = -(C.st2pi * (sxv * syv)) - C.ct * lwr[(i & (K - 1)) * W + lane];
        acc[c + E] = fma(qs, b, acc[c + E]);
      }
      // pin the adds of the last PIN rows before the next row's DMA / wait / LDS
      // reads: unpinned, the compiler sinks them and keeps many rows' windows
      // live (spills); pinned every PIN rows, PIN rows' dependency chains
      // (the nested-window core) interleave
      if constexpr (c % PIN == PIN - 1) {
#pragma unroll
        for (int a = c + 1 - PIN; a <= c + 2 * E; ++a) asm volatile("" : "+v"(acc[a]));
      }
    };
    static_for<CH>(row);
    // outputs a = 0 .. CH-1 complete: k = ibase - 2E + a
    full = ibase - 2 * E >= 0 && ibase - 2 * E + CH <= nout;
    // SP: one 64-bit row multiply per chunk; the CH stores step a row pointer
    // (ISA: 19 scalar instructions per store with the multiply each, E = 32)
    double *op = SP ? run + (int64_t)(up ? Y1 - 1 - (ibase - 2 * E) : Y0 + (ibase - 2 * E)) * pitch : nullptr;
    auto store = [&](auto ac) __attribute__((always_inline)) {
      constexpr int a = decltype(ac)::value;
      const int k = ibase - 2 * E + a;
      double *const orow = op;
      if constexpr (SP) op += stride;
      if (k < 0 || k >= nout) return;
      if (emit) {
        double *dst = SP ? orow + xl : run + (int64_t)(up ? Y1 - 1 - k : Y0 + k) * pitch + xl;
        if constexpr (NTS)
          __builtin_nontemporal_store(alpha * acc[a], dst);  // NTS: streaming store (tools/ harness)
        else
          *dst = alpha * acc[a];
      }
    };
    static_for<CH>(store);
    // rename: a -> a - CH
#pragma unroll
    for (int a = 0; a < 2 * E; ++a) acc[a] = acc[a + CH];
  }
  wait_vmcnt<0>();  // drain the clamped tail DMAs and the stores
}

// rows per chunk: 12 up to E = 32; 8 beyond, where the 2E + CH accumulators
// fill the 256 arch VGPRs (E = 40: 256, E = 48: 274 with AGPRs, no scratch;
// one wave per SIMD past E = 40)
template <int E>
constexpr int wide_chunk() { return E <= 32 ? kWideC : 8; }

// prefix-sum row windows where they keep k_wide within the 256 VGPRs of two
// waves per SIMD (hipcc 7.2, 8-row chunks past 32: 240 / 248 / 256 at E = 33 /
// 34 / 35, 260+ from 36): C4 at 8192^2 143 vs 128 G node/s, eps 33 113 vs
// 108 G.  Past that the two-chunk scan costs the second wave: eps 40 71 vs
// 102 G, eps 48 54 vs 66 G (profiles/r02/evidence/wide_ps/) -- nested sums
template <int E>
constexpr bool wide_ps() { return E <= 35; }

// prefix-sum rows (E <= 35) are built two rows ahead of their window reads,
// each read a separate ds_read_b64, in 8-row chunks: C4 (8192^2, eps 32)
// 139.5 -> 155.8 G node/s in tools/wide_bench.hip, bitwise equal
// (profiles/r03/wide_pa_sweep.jsonl)
// (E <= 32: 146-251 VGPRs, two waves per SIMD; at 33-35 the prefetched
// windows would take 256-274 and one wave per SIMD, so those keep PA = 0)
template <int E>
constexpr int wide_pa() { return E <= 32 ? 2 : 0; }
template <int E>
constexpr int wide_chunk_pa() { return E <= 32 ? 8 : wide_chunk<E>(); }
// ... with the scan interleaved into the taps (ILS): C4 153.4-155.6 ->
// 156.9-157.6 G node/s in tools/wide_bench.hip, bitwise equal
// (profiles/r03/wide_ils.jsonl); and non-temporal output stores (NTS, the
// same instances): +1-2% (profiles/r03/wide_nts.jsonl)
template <int E>
constexpr bool wide_ils() { return wide_pa<E>() > 0; }

// ... and row pairs (RP) in production: C4 159.0 -> 165.4-167.0 G node/s in
// tools/wide_bench.hip (profiles/r03/rowpairs/wide_rp.jsonl; 248 -> 254 VGPRs,
// two waves per SIMD), and on the nested windows past E = 40 (one wave per
// SIMD there either way): eps 48 67.1 -> 67.5-67.9, eps 64 36.3 -> 39.7 G
// (profiles/r03/rowpairs/wide{48,64}.jsonl).  E = 33..40 keep one-row taps
// (two waves per SIMD at up to 256 VGPRs without them).  Test mode keeps RP
// off: at E = 32 its source terms push RP past 256 VGPRs (one wave per SIMD)
template <int E, bool TEST>
constexpr bool wide_rp() { return !TEST && (wide_pa<E>() > 0 || E > 40); }

// ... and the chunk's output row pointer (SP) instead of a 64-bit row multiply
// per store: C4 398-402 -> 391-397 us per step in tools/wide_bench.hip, bitwise
// equal, same registers at every E (profiles/r04/widesp)
template <int E, bool TEST>
int launch_wide_e(const RectList &rl, const StepConst &c, hipStream_t st) {
  hipLaunchKernelGGL((k_wide<E, wide_chunk_pa<E>(), TEST, kWideD, 0, 1, false, 16, true, wide_ps<E>(), wide_pa<E>(),
                             (wide_pa<E>() > 0), wide_ils<E>(), wide_ils<E>(), wide_rp<E, TEST>(), true>),
                     dim3(rl.nwork), dim3(64), 0, st, rl, c);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// resident k_wide workgroups (one wave each) per CU, for the host's choice of
// segment height
template <int E>
int wide_blocks_per_cu_e() {
  int n = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &n, k_wide<E, wide_chunk_pa<E>(), false, kWideD, 0, 1, false, 16, true, wide_ps<E>(), wide_pa<E>(),
             (wide_pa<E>() > 0), wide_ils<E>(), wide_ils<E>(), wide_rp<E, false>(), true>,
      64, 0);
  return e == hipSuccess ? n : 0;
}

}  // namespace nlh
