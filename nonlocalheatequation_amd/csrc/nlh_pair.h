// nlh_pair.h -- two explicit-Euler steps per pass over HBM (temporal
// blocking of the reference's do_work loop, src/2d_nonlocal_serial.cpp:273-303:
// u^{t+1} = u^t + dt*L_h[u^t] applied twice, production mode, no source term).
//
// One 64-lane wave per (strip, segment), like k_fast (nlh_fast.h), but every
// u^t row streamed HBM -> LDS feeds TWO nested-window sweeps:
//
//   stage 1: u^{t+1} over the 64*R columns x0-E .. x0-E+64R (the strip plus an
//            E-wide halo on both sides), rows Y0-E .. Y1+E; values outside the
//            lattice are forced to 0 (the reference's zero boundary) and each
//            finished row is written to one of two LDS row buffers;
//   stage 2: the same sweep over those u^{t+1} rows, one row behind stage 1,
//            emitting u^{t+2} for the 64R-2E columns x0 .. x0+64R-2E and rows
//            Y0 .. Y1.
//
// u^{t+1} never touches HBM: per two steps the kernel reads u^t (with a 2E
// halo) and writes u^{t+2} once, about half the single-step traffic.
//
// Nested windows with a shared core.  A lane owns two adjacent columns a, b
// and reads the 2E+2 values w[0..2E+1] around them.  With the core
// K_L = w[E+1-L] + .. + w[E+L]:  H_L(a) = K_L + w[E-L],  H_L(b) = K_L + w[E+1+L],
// evaluated only at the levels L the disk uses; 2E-1 + 2*levels adds per row
// instead of 4E (25 instead of 32 at E = 8).  The accumulator of the output
// E rows ahead receives its first term from this row (level 0, d = +E), so it
// is assigned and never has to be zeroed.
//
// Centre fold: u' = u + alpha*(S - N u) = alpha*(S + (1/alpha - N) u), so the
// centre value is added to its own accumulator (kc = 1/alpha - N) when its row
// arrives and no centre rows have to be kept.  The extra rounding is a few ulp
// of the field scale; alpha == 0 never reaches this kernel.
//
// Iteration i: DMA u^t row i+D -> wait for row i -> ds_read the u^{t+1}
// window of row i-2E-1 (written by the previous iteration) and the u^t
// window of row i -> stage-2 math (covers the LDS latency of the u^t window)
// -> stage-1 math -> ds_write u^{t+1} row i-2E.  No LDS write->read round
// trip sits on the critical path.
#pragma once

#include "nlh_device.h"
#include "nlh_kernel_common.h"

namespace nlh {

constexpr int kPairSplitD = 8;  // k_pair_split: rows in flight beyond the next block
constexpr int kPairSplitB = 4;  // k_pair_split: rows per barrier
// k_pair_split code-shape and scheduling options (results bitwise identical): 1 = the output
// row pointer advances by one row per iteration (no 64-bit row multiply and
// fewer scalar instructions per store); 2 = unclamped row DMA (the ring's
// tail DMAs, at most 2B + D rows past a segment's last input row, read the
// kPairPadRows padding rows the host allocates beyond each block's halo rows
// for pair passes); 4 = the single-column store of an odd-width rect's last
// lane behind a wave-uniform test.  C2 harness (profiles/r04/{pairopt,
// eighth,pairopt2}): per pass 75.8 us with none, 74.3-75.5 with 1, 74.7-75.3
// with 1 + 4, 74.0-75.0 with all three.  E = 13 leaves out 1: with it hipcc
// 7.2 allocates 256 VGPRs and spills 76-116 bytes there (229 / 242 without).
// 8 = wave 1 (DMA + stage 2 + stores, the longer of the two lockstep roles)
// at wave priority 3 (s_setprio), so a SIMD holding it beside another
// workgroup's stage-1 wave issues it first: C2 harness 73.3-74.9 -> 71.5-72.8
// us per pass, bitwise equal (priority 1 / 2: 71.7-73.0 / 72.3-72.7;
// wave 0 first instead: 73.5-74.1; profiles/r04/prio/)
// 16 = the head taps left out: the first period of each stage is peeled, and
// there a row's taps into output rows that are never emitted (i+d < E) and
// the nested-window levels only those taps use are skipped (pair_scatter LO;
// 3.4% fewer f64 adds at C2).  32 = a barrier block's first row also reads
// the second row's window (B == 2, even period).  64 = 32 and the two rows of
// a pair build their nested windows in one interleaved instruction stream
// (pair_levels2 / pair_taps).  All bitwise equal.  C2 harness, the variants
// interleaved ten times over on one box (profiles/r05/pair_opt/): median per
// pass 72.48 us (15), 70.41 (15|16|32), 73.37 (15|64), 69.67 (15|16|64).
// 32 / 64 need ~30 more VGPRs: hipcc spills at E = 13, 14 (test mode), 16,
// so those take 16 alone; E = 1, 2 have no row pairs.  128 = the tail rows
// likewise (pair_tail_c: segments of the C2 height only, E = 8), 256 = the
// stage-1 periods between head and tail without per-row tests (lean).  Where
// the time goes at C2 (profiles/r05/): eight extra s_nop per row cost 2.4% on
// the stage-1 wave and nothing on the stage-2 wave -- wave 0 is the critical
// role under the wave priority, so work off its path pays.  Medians over
// interleaved repetitions on one box: 15|16|64|128 69.84 us, |256 68.53
// (E = 8 only: measured there; the lean stage 2 makes hipcc spill).  2048 =
// rings whose slot counts divide the period (production; E = 8: 27.7 KB of
// LDS per workgroup, 4 per CU): 67.62 -> 66.44 us (profiles/r05/pair/ring_*).
// 512 (harness only) puts wave 0 at the wave priority instead of wave 1;
// 1024 (harness only) the lean stage 2 (spills).  32768 (test mode, E = 8;
// off): the L_h[W0] rows from the separable form L_h[W0] = sum_l Sx'_l(x)
// Ty_l(y) + sx(x) Z(y) (StepConst lsx / lty) -- per row a 64-byte Ty / Z DMA
// instead of the 1-KB L_h[W0] row, wave 1 forming the row B iterations ahead
// of wave 0: C2 test-mode harness 98.9 -> 94.7 us per pass, 4.4e-16 from the
// field (profiles/r05/pair/test_sep2_reps4.jsonl), but in the library build
// 96.5 -> 103.9 us per pass (rocprofv3, 51.1 vs 46.0 VALU lane-ops per
// node-update; profiles/r05/evidence_2c33717e/test), so the library keeps
// the L_h[W0] row DMA.
constexpr int kPairPadRows = 16;
__host__ __device__ constexpr bool pair_rows(int E);
__host__ __device__ constexpr int pair_opt(int E) {
  return E == 8 ? 15 | 16 | 64 | 128 | 256 | 2048 | 4096
                : (E == 13 ? 14 | 16 : (E <= 12 && pair_rows(E) ? 15 | 16 | 64 : 15 | 16));
}

// separable L_h[W0] (OPT & 32768): the distinct half-widths L > 0 of the disk
// rows in order of first appearance (d = 0, 1, ..), their count NLV, and the
// row stride of the per-row table (NLV values + Z, a power of two)
__host__ __device__ constexpr int pair_sep_level(int E, int l) {
  int k = 0, prev = -1;
  for (int d = 0; d <= E; ++d) {
    const int L = clen(E, d);
    if (L > 0 && L != prev) {
      if (k == l) return L;
      ++k;
    }
    prev = L;
  }
  return -1;
}
__host__ __device__ constexpr int pair_sep_nlv(int E) {
  int n = 0;
  while (pair_sep_level(E, n) > 0) ++n;
  return n;
}
__host__ __device__ constexpr int pair_sep_stride(int E) { return pair_sep_stride_n(pair_sep_nlv(E)); }

// some row offset d of the disk has half-width len(d) == L
__host__ __device__ constexpr bool pair_level_used(int E, int L) {
  for (int d = 0; d <= E; ++d)
    if (clen(E, d) == L) return true;
  return false;
}

// Row pairs.  Rows are scattered in pairs, A (even row) then B (the next
// row).  Where the disk's half-width is the same at two adjacent row offsets,
// len(d) == len(d-1) > 0, the output row o = A + d receives H_L(A) (offset d)
// and H_L(B) (offset d-1) of the same level L: row A skips that tap and row B
// adds the pair sum H_L(A) + H_L(B) once -- one extra add per shared level
// serves every such offset.  E = 8: offsets -4, -2, -1, 2, 3, 5 (levels 6 and
// 7), 4 adds fewer per row pair and column (30 instead of 34).
__host__ __device__ constexpr int pair_abs(int d) { return d < 0 ? -d : d; }
__host__ __device__ constexpr bool pair_shared(int E, int d) {
  return d > -E && d <= E && clen(E, pair_abs(d)) > 0 && clen(E, pair_abs(d)) == clen(E, pair_abs(d - 1));
}
__host__ __device__ constexpr bool pair_level_shared(int E, int L) {
  for (int d = -E; d <= E; ++d)
    if (pair_shared(E, d) && clen(E, pair_abs(d)) == L) return true;
  return false;
}
__host__ __device__ constexpr bool pair_rows(int E) {
  for (int d = -E; d <= E; ++d)
    if (pair_shared(E, d)) return true;
  return false;
}
// accumulator slots: the 2E+1 output rows a row touches, one more with row
// pairs so that the unrolled period is even and no pair straddles it
__host__ __device__ constexpr int pair_slots(int E) { return pair_rows(E) ? 2 * E + 2 : 2 * E + 1; }

// window of 2E+R values starting at p (16-B aligned) into w
template <int E, int R>
__device__ __forceinline__ void pair_window(const double *p, double (&w)[R + 2 * E]) {
  constexpr int NB = (R + 2 * E + 1) / 2;
  const double2 *rp = reinterpret_cast<const double2 *>(p);
  double buf[2 * NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const double2 v = rp[k];
    buf[2 * k] = v.x;
    buf[2 * k + 1] = v.y;
  }
#pragma unroll
  for (int k = 0; k < R + 2 * E; ++k) w[k] = buf[k];
}

// Nested windows of the lane's two columns scattered into the accumulators
// of the 2E+1 output rows this input row touches (slot of output row
// input+d = (QA + d) mod P; QA = the input row's own slot), plus the folded
// centre term.  ROLE 0: a lone row (no row pairs at this E); 1: row A of a
// pair (shared taps left to B, its shared levels kept in hs); 2: row B (the
// pair sums at the shared taps).
// LO (head rows of a segment, OPT & 16): taps at offsets d < LO go to output
// rows that are never emitted and are left out, and the nested windows are
// built only up to the largest level a kept tap uses.
// HI (tail rows of a segment, OPT & 128): likewise for taps at offsets d > HI
template <int E, int LO, int HI = E>
__host__ __device__ constexpr int pair_head_lmax() {
  int m = -1;
  for (int d = (LO < -E ? -E : LO); d <= (HI > E ? E : HI); ++d)
    m = clen(E, pair_abs(d)) > m ? clen(E, pair_abs(d)) : m;
  return m;
}

template <int E, int QA, int ROLE, int LO = -E, int HI = E>
__device__ __forceinline__ void pair_scatter(const double (&w)[2 * E + 2], double (&acc)[2][pair_slots(E)],
                                             double kc, double (&hs)[2][E + 1]) {
  constexpr int P = pair_slots(E);
  constexpr int SF = (QA + E) % P;      // d = +E: first term of that output row
  constexpr int SL = (QA + P - E) % P;  // d = -E: last term
  constexpr int LMAX = pair_head_lmax<E, LO, HI>();
  if constexpr (E >= LO && E <= HI) {
    acc[0][SF] = w[E];
    acc[1][SF] = w[E + 1];
  }
  if constexpr (-E >= LO && -E <= HI) {
    acc[0][SL] += w[E];
    acc[1][SL] += w[E + 1];
  }
  // levels and taps are template constants (static_for): evaluating the
  // disk shape inside the row loop at run time costs more than the sums
  double core = w[E] + w[E + 1];
  auto level = [&](auto lc) {
    constexpr int Lv = decltype(lc)::value + 1;
    if constexpr (Lv > 1 && Lv <= LMAX) core = core + (w[E + 1 - Lv] + w[E + Lv]);
    if constexpr (pair_level_used(E, Lv) && Lv <= LMAX) {
      const double ha = core + w[E - Lv];
      const double hb = core + w[E + 1 + Lv];
      constexpr bool shl = ROLE != 0 && pair_level_shared(E, Lv);
      double pa = ha, pb = hb;
      if constexpr (shl && ROLE == 1) {
        hs[0][Lv] = ha;
        hs[1][Lv] = hb;
      } else if constexpr (shl && ROLE == 2) {
        pa = hs[0][Lv] + ha;
        pb = hs[1][Lv] + hb;
      }
      auto tap = [&](auto dc) {
        constexpr int d = decltype(dc)::value - E;
        constexpr int s = (QA + d + P) % P;
        if constexpr (clen(E, pair_abs(d)) == Lv && d >= LO && d <= HI) {
          if constexpr (ROLE == 1 && pair_shared(E, d)) {
            // row B adds the pair sum
          } else if constexpr (ROLE == 2 && pair_shared(E, d + 1)) {
            acc[0][s] += pa;
            acc[1][s] += pb;
          } else {
            acc[0][s] += ha;
            acc[1][s] += hb;
          }
        }
      };
      static_for<2 * E + 1>(tap);
    }
  };
  static_for<E>(level);
  if constexpr (0 >= LO && 0 <= HI) {
    acc[0][QA] = fma(kc, w[E], acc[0][QA]);
    acc[1][QA] = fma(kc, w[E + 1], acc[1][QA]);
  }
}

// OPT & 64: pair_scatter split in two, so that the nested windows of the two
// rows of a pair are built in ONE instruction stream (two independent
// dependency chains of core adds interleaved) before row A's taps; row B's
// taps follow one row later.  Same adds in the same order per value as
// pair_scatter: bitwise equal results.
//   hv[L][c]: H_L of the lane's column c (c = 0: a, 1: b) at every used level
template <int E, int LMAX>
__device__ __forceinline__ void pair_levels(const double (&w)[2 * E + 2], double (&hv)[E + 1][2]) {
  double core = w[E] + w[E + 1];
  static_for<E>([&](auto lc) __attribute__((always_inline)) {
    constexpr int Lv = decltype(lc)::value + 1;
    if constexpr (Lv > 1 && Lv <= LMAX) core = core + (w[E + 1 - Lv] + w[E + Lv]);
    if constexpr (pair_level_used(E, Lv) && Lv <= LMAX) {
      hv[Lv][0] = core + w[E - Lv];
      hv[Lv][1] = core + w[E + 1 + Lv];
    }
  });
}

template <int E, int LMA, int LMB>
__device__ __forceinline__ void pair_levels2(const double (&wa)[2 * E + 2], const double (&wb)[2 * E + 2],
                                             double (&ha)[E + 1][2], double (&hb)[E + 1][2]) {
  double ca = wa[E] + wa[E + 1];
  double cb = wb[E] + wb[E + 1];
  static_for<E>([&](auto lc) __attribute__((always_inline)) {
    constexpr int Lv = decltype(lc)::value + 1;
    if constexpr (Lv > 1 && Lv <= LMA) ca = ca + (wa[E + 1 - Lv] + wa[E + Lv]);
    if constexpr (Lv > 1 && Lv <= LMB) cb = cb + (wb[E + 1 - Lv] + wb[E + Lv]);
    if constexpr (pair_level_used(E, Lv) && Lv <= LMA) {
      ha[Lv][0] = ca + wa[E - Lv];
      ha[Lv][1] = ca + wa[E + 1 + Lv];
    }
    if constexpr (pair_level_used(E, Lv) && Lv <= LMB) {
      hb[Lv][0] = cb + wb[E - Lv];
      hb[Lv][1] = cb + wb[E + 1 + Lv];
    }
  });
}

// the taps of pair_scatter from precomputed levels hv (this row) and hA (row
// A's, for row B's pair sums)
template <int E, int QA, int ROLE, int LO = -E, int HI = E>
__device__ __forceinline__ void pair_taps(const double (&w)[2 * E + 2], const double (&hv)[E + 1][2],
                                          const double (&hA)[E + 1][2], double (&acc)[2][pair_slots(E)],
                                          double kc) {
  constexpr int P = pair_slots(E);
  constexpr int SF = (QA + E) % P;
  constexpr int SL = (QA + P - E) % P;
  if constexpr (E >= LO && E <= HI) {
    acc[0][SF] = w[E];
    acc[1][SF] = w[E + 1];
  }
  if constexpr (-E >= LO && -E <= HI) {
    acc[0][SL] += w[E];
    acc[1][SL] += w[E + 1];
  }
  static_for<E>([&](auto lc) __attribute__((always_inline)) {
    constexpr int Lv = decltype(lc)::value + 1;
    if constexpr (pair_level_used(E, Lv)) {
      static_for<2 * E + 1>([&](auto dc) __attribute__((always_inline)) {
        constexpr int d = decltype(dc)::value - E;
        constexpr int s = (QA + d + P) % P;
        if constexpr (clen(E, pair_abs(d)) == Lv && d >= LO && d <= HI) {
          if constexpr (ROLE == 1 && pair_shared(E, d)) {
            // row B adds the pair sum
          } else if constexpr (ROLE == 2 && pair_shared(E, d + 1)) {
            acc[0][s] += hA[Lv][0] + hv[Lv][0];
            acc[1][s] += hA[Lv][1] + hv[Lv][1];
          } else {
            acc[0][s] += hv[Lv][0];
            acc[1][s] += hv[Lv][1];
          }
        }
      });
    }
  });
  if constexpr (0 >= LO && 0 <= HI) {
    acc[0][QA] = fma(kc, w[E], acc[0][QA]);
    acc[1][QA] = fma(kc, w[E + 1], acc[1][QA]);
  }
}

// tap bounds of one row of a pass (LO, HI) and of the next row (PI: the
// pair's row B, whose levels row A builds)
// LEAN_ (OPT & 256): a row of a period known to lie wholly inside the
// segment's rows and the lattice, past the warm-up -- no per-row range,
// emission or lattice-edge tests and the barrier placement a template
// constant (B divides the period), so the period runs without branches
template <int LO_, int HI_, int LON_, int HIN_, bool LEAN_ = false>
struct PairRowBounds {
  static constexpr int LO = LO_, HI = HI_, LON = LON_, HIN = HIN_;
  static constexpr bool LEAN = LEAN_;
};

// OPT & 128: the tail rows of a segment skip their taps into output rows that
// are never emitted, like the head (OPT & 16) -- possible where the last
// period's slots are template constants, i.e. when the segment's u^t row
// count n_in = seg + 4E is congruent to pair_tail_c(E) modulo the period: the
// host's one-round segment height at 4096^2 (C2; nlh_api.cpp sizes()).  Other
// segments take the generic loop.  Stage 1's tail is its last X1 rows, stage
// 2's its last X2 iterations (each >= 2E, the period-aligned end).
__host__ __device__ constexpr int pair_tail_c(int E) {
  // (seg + 4E) mod period at the C2 segment height of each E
  return E == 8 ? 4 : -1;
}
// the least divisor of P that is >= lo (OPT & 2048's u^{t+1} ring)
__host__ __device__ constexpr int pair_ring_divisor(int P, int lo) {
  for (int d = lo; d <= P; ++d)
    if (P % d == 0) return d;
  return P;
}
__host__ __device__ constexpr int pair_tail_len(int E, int c) {
  const int P = pair_slots(E);
  int x = ((c % P) + P) % P;
  while (x < 2 * E) x += P;
  return x;
}

// ABL: timing-decomposition masks for the tools/ harness (tools/pair_bench.hip).
// 4096 / 8192: eight extra s_nop per row on wave 0 / wave 1 (the cost of
// non-VALU instructions on each role's path).
// libnlh instantiates ABL = 0 only (tests/test_capi.py checks the library's
// kernel symbols); with ABL != 0 the results are meaningless.  k_pair_split:
// 2 = no HBM traffic (no DMA, no stores; same instruction stream otherwise),
// 4 = windows from registers (no LDS window reads), 8 = no s_barrier,
// 16 = no u^{t+1} LDS writes, 32 = no per-row range checks (rows past the
// segment end computed too), 64 = no vmcnt waits for the DMA'd rows, 128 = no
// output stores, 256 = no DMA, 512 = non-temporal stores, 1024 = non-temporal DMA,
// 16384 = (test mode) no L_h[W0] row DMA

// k_pair_split: the two stages of k_pair on the two waves of one workgroup,
// synchronised once per block of B rows (s_barrier):
//   wave 0 (stage 1): u^t row i from the LDS ring -> u^{t+1} row i-2E into a
//                     2B-row LDS ring;
//   wave 1 (memory + stage 2): LDS-DMA of u^t row i+B+D (and, at each block
//                     end, the wait for the next block's rows, so wave 0
//                     never waits on HBM), stage 2 on u^{t+1} row i-2E-B (the
//                     block wave 0 finished before the last barrier), and the
//                     u^{t+2} store.
// Each wave holds ONE accumulator set (2 x (2E+1) doubles): at the two waves
// per SIMD of k_pair a workgroup owns a segment twice as tall, so less of the
// 4E / 2E rows of redundant halo work per segment (4 workgroups per CU
// measured best, see nlh_api.cpp); one barrier per B rows lets per-row
// jitter of the two waves average out.  Same arithmetic and order as
// k_pair: bitwise equal results.
//
// TEST (manufactured source, sum_local_test :235-252, in the fast form
// b(x,t) = -(2 pi st_t) W0(x) - ct_t L_h[W0](x) with the precomputed plane
// L_h[W0] of k_fast): wave 1 also DMAs, with u^t row i, the L_h[W0] row and
// the sin(2 pi y dh) entry of u^{t+1} row i-2E.  Stage 1 adds dt*b(t) to
// u^{t+1} and writes (dt/alpha)*b(t+1) beside it into a second 2B-row ring;
// stage 2 folds that into the centre accumulator of the same row, so
// u^{t+2} = alpha*(S + kc u^{t+1} + (dt/alpha) b(t+1)).  L_h[W0] is read once
// per two steps.
template <int E, int D, int ABL = 0, int B = kPairSplitB, bool TEST = false, int OPT = pair_opt(E)>
__global__ __launch_bounds__(128, 2) void k_pair_split(RectList L, StepConst C) {
  constexpr int R = 2;
  constexpr int P = pair_slots(E);      // accumulator slots = rows per unrolled period
  constexpr bool PAIRS = (P & 1) == 0;  // rows scattered in pairs (even row = A)
  constexpr int W1 = 64 * R;
  constexpr int WO = W1 - 2 * E;
  constexpr int NW = R + 2 * E;
  constexpr int RW = W1 + 2 * E;
  constexpr int NCH = RW / 2;
  constexpr int DT = B + D;             // rows fetched ahead of wave 0's row
  // OPT & 2048 (production): rings whose slot counts divide the period, so
  // every period starts at slot 0 and a row's ring slots are template
  // constants (LDS offsets in the instructions, no slot arithmetic per row):
  // the u^t ring holds one period (K = P >= DT + B rows), the u^{t+1} ring the
  // least divisor of P that holds its 2B live rows
  constexpr bool RP = (OPT & 2048) != 0 && !TEST && P >= DT + B;
  constexpr int K = RP ? P : pow2_ceil(DT + B);  // rows i .. i+DT+B-1 live at once
  constexpr int G = (NCH + 63) / 64;
  constexpr int U1W = W1 + 2 * E + 2;
  constexpr int U1R = RP ? pair_ring_divisor(P, 2 * B) : 2 * B;  // u^{t+1} ring rows
  // TEST: L_h[W0] row of the stage-1 columns x0-E .. x0-E+W1-1, staged from
  // the even column at or before x0-E (16-byte DMA chunks)
  constexpr int LOFF = E & 1;
  constexpr int NCHL = TEST ? (W1 + LOFF + 1) / 2 : 0;
  constexpr int LWW = 2 * NCHL;
  // OPT & 32768 (test mode): L_h[W0] rows formed by wave 1 from the
  // separable tables (StepConst lsx / lty) instead of read from HBM
  constexpr bool SEP = TEST && (OPT & 32768) != 0;
  constexpr int NLV = SEP ? pair_sep_nlv(E) : 0;
  constexpr int LTS = SEP ? pair_sep_stride(E) : 0;
  // SEP: one DMA per row for the row's Ty / Z values (LTS doubles) instead of its L_h[W0] row
  constexpr int GT = TEST ? (SEP ? 1 : (NCHL + 63) / 64) + 1 : 0;  // + the sin(2 pi y dh) pair
  constexpr int GA = G + GT;            // DMA instructions per row
  static_assert((B & (B - 1)) == 0, "B must be a power of two");
  static_assert(D * GA + D + 1 < 64, "vmcnt range");
  static_assert(WO >= 64, "strip too narrow for this eps");
  static_assert(P <= 2 * E + B, "the peeled iterations 0 .. P-1 carry no u^{t+1} row");
  static_assert((OPT & 2) == 0 || 2 * B + D <= kPairPadRows, "tail DMAs past the padding rows");

  __shared__ __attribute__((aligned(16))) double ring[K * RW + U1R * U1W + (TEST ? U1R * U1W + K * LWW + 2 * K : 0) +
                                                     K * LTS];
  double *const u1buf = ring + K * RW;
  double *const qbuf = u1buf + U1R * U1W;  // TEST: (dt/alpha) b(t+1) of the u^{t+1} rows
  double *const lwr = qbuf + U1R * U1W;    // TEST: L_h[W0] rows, slots of the u^t ring
  double *const syr = lwr + K * LWW;       // TEST: sin(2 pi y dh) pairs, same slots
  [[maybe_unused]] double *const tyr = syr + 2 * K;  // SEP: Ty / Z rows, same slots
  // ring slots: bsv = b mod K (0 with RP), q = the row's place in the period
  auto kslot = [](int bsv, int q) __attribute__((always_inline)) { return RP ? q % K : (bsv + q) & (K - 1); };
  auto uslot = [](int m, int qm) __attribute__((always_inline)) {
    return RP ? ((qm % U1R) + U1R) % U1R : m & (U1R - 1);
  };

  const int lane = (int)(threadIdx.x & 63);
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &Rc = L.r[ri];
  const int rx1 = Rc.x1, rgx0 = Rc.gx0, rgy0 = Rc.gy0;
  const int local = work - Rc.wg_begin;
  const int nstrip = Rc.nstrip;
  const int strip = local % nstrip, seg = local / nstrip;
  const int x0 = Rc.x0 + strip * WO;
  const int seg_h = Rc.seg_rows;
  const int Y0 = Rc.y0 + seg * seg_h;
  const int Y1 = min(Y0 + seg_h, Rc.y1);
  const int n_in = (Y1 - Y0) + 4 * E;   // u^t rows Y0-2E .. Y1+2E-1
  const int i_last = n_in - 1 + B;      // wave 1's last iteration
  const bool up = (seg & 1) != 0;
  const int64_t pitch = Rc.pitch;
  const int64_t stride = up ? -pitch : pitch;
  const double alpha = C.alpha, kc = C.kc;
  const int ydir = up ? -1 : 1;
  // TEST: block row of u^{t+1} row m (clamped to the rows a segment computes)
  // and the sin(2 pi y dh) table index of that row
  const int nm = n_in - 2 * E;
  auto m_row = [&](int m) {
    m = min(max(m, 0), nm - 1);
    return up ? (Y1 + E - 1 - m) : (Y0 - E + m);
  };
  auto sy_idx = [&](int m) { return min(max(rgy0 + m_row(m) + E, 0), (int)C.ny + 2 * E - 1); };

  // s_barrier with every LDS access of this wave completed first; the asm
  // "memory" clobber also keeps the compiler from moving LDS accesses across
  auto row_barrier = [] {
    if constexpr ((ABL & 8) != 0)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ablation: no s_barrier
    else
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  // ablation ABL & 4: windows from registers instead of LDS (opaque values)
  auto window = [&](const double *p, double (&w)[NW]) {
    if constexpr ((ABL & 4) != 0) {
#pragma unroll
      for (int k = 0; k < NW; ++k) {
        w[k] = (double)(lane + k);
        asm volatile("" : "+v"(w[k]));
      }
    } else {
      pair_window<E, R>(p, w);
    }
  };

  double acc[R][P];
#pragma unroll
  for (int c = 0; c < R; ++c)
#pragma unroll
    for (int j = 0; j < P; ++j) acc[c][j] = 0.0;
  double hs[R][E + 1];  // row A's windows at the shared levels, until row B
  constexpr bool PF = ((OPT & 32) != 0 || (OPT & 64) != 0) && B == 2 && (P & 1) == 0;
  constexpr bool PI = (OPT & 64) != 0 && PF && PAIRS;  // row pairs' levels interleaved
  double wr[2][NW];     // the row's window (and, PF, the next row's)
  [[maybe_unused]] double hv[2][E + 1][2];  // PI: the levels of a pair's rows A, B

  // ABL & 2048 (tools/pair_bench.hip only): per wave, HW_ID, XCC_ID and the
  // s_memrealtime stamps at entry and exit into the uint64 buffer at Rc.lw
  [[maybe_unused]] uint64_t t_entry = 0;
  if constexpr ((ABL & 2048) != 0) t_entry = __builtin_amdgcn_s_memrealtime();
  if constexpr ((OPT & 8) != 0)
    if (wave == ((OPT & 512) != 0 ? 0 : 1)) __builtin_amdgcn_s_setprio(3);
  if (wave == 0) {
    // ---- stage 1 on u^t row i
    const int gny = (int)C.ny;
    const int gy1first = rgy0 + (up ? (Y1 + E - 1) : (Y0 - E));
    double mcol[R], sxv[R];
#pragma unroll
    for (int c = 0; c < R; ++c) {
      const int gx = rgx0 + x0 - E + R * lane + c;
      mcol[c] = (gx >= 0 && gx < (int)C.nx) ? alpha : 0.0;
      sxv[c] = TEST ? C.sxt[min(max(gx, -E), (int)C.nx + E - 1) + E] : 0.0;
    }
    const double qs = TEST ? C.dt / alpha : 0.0;
    row_barrier();  // prologue: rows 0 .. B-1 landed
    int bs = 0;     // b % K
    // OPT & 16: the first period (rows 0 .. P-1) peeled with the head taps
    // of pair_scatter left out (row i's outputs i+d < E are never emitted);
    // OPT & 128: the last X1 rows likewise (outputs i+d >= n_in - E)
    constexpr bool HEAD = (OPT & 16) != 0;
    int b = 0;
    auto body = [&](auto qc, auto bc) __attribute__((always_inline)) {
        constexpr int q = decltype(qc)::value;
        using RB = decltype(bc);
        constexpr int LO = RB::LO, HI = RB::HI;
        constexpr int so = (q + P - E) % P;  // output row i - E completes
        const int i = b + q;
        if constexpr ((ABL & 32) == 0 && !RB::LEAN)
          if (i >= n_in) return;
        // OPT & 32 (B == 2 and an even period, so a row's place in its barrier
        // block is a template constant): a block's first row also reads the
        // second row's window, which the last barrier already published
        double (&w)[NW] = wr[q & 1];
        if constexpr (!PF || (q & 1) == 0) window(ring + kslot(bs, q) * RW + R * lane, w);
        if constexpr (PF && (q & 1) == 0) window(ring + kslot(bs, q + 1) * RW + R * lane, wr[1]);
        if constexpr (PI) {
          if constexpr ((q & 1) == 0)
            pair_levels2<E, pair_head_lmax<E, LO, HI>(), pair_head_lmax<E, RB::LON, RB::HIN>()>(wr[0], wr[1],
                                                                                               hv[0], hv[1]);
          pair_taps<E, q, 1 + (q & 1), LO, HI>(w, hv[q & 1], hv[0], acc, kc);
        } else {
          pair_scatter<E, q, PAIRS ? 1 + (q & 1) : 0, LO, HI>(w, acc, kc, hs);
        }
        if (RB::LEAN || (ABL & 32) != 0 || i >= 2 * E) {
          const int m = i - 2 * E;
          const int gy = gy1first + ydir * m;
          double v0 = mcol[0] * acc[0][so];
          double v1 = mcol[1] * acc[1][so];
          double q0 = 0.0, q1 = 0.0;
          if constexpr (TEST) {
            const int slot = kslot(bs, q);  // u^t row i: its L_h[W0] / sin rows
            const double syv = syr[2 * slot + (sy_idx(m) & 1)];
            const double *lrow = lwr + slot * LWW + LOFF + R * lane;
            const double w00 = sxv[0] * syv, w01 = sxv[1] * syv;
            const double lw0 = lrow[0], lw1 = lrow[1];
            v0 = fma(-(C.st2pi * w00) - C.ct * lw0, C.dt, v0);
            v1 = fma(-(C.st2pi * w01) - C.ct * lw1, C.dt, v1);
            q0 = qs * (-(C.st2pi2 * w00) - C.ct2 * lw0);
            q1 = qs * (-(C.st2pi2 * w01) - C.ct2 * lw1);
            if (mcol[0] == 0.0) v0 = 0.0;  // columns outside the lattice
            if (mcol[1] == 0.0) v1 = 0.0;
          }
          if constexpr (RB::LEAN) {
            // lean rows: a select (v_cndmask on a wave-uniform condition), no
            // branch.  OPT & 4096: only the first 3E - P rows of a period take
            // it -- a lean period starts at b >= P, so its rows q >= 3E - P lie
            // past the segment's first E u^{t+1} rows, and lean periods end
            // before its last E (the only rows that can leave the lattice)
            if constexpr ((OPT & 4096) == 0 || q < 3 * E - P) {
              const bool out = gy < 0 || gy >= gny;
              v0 = out ? 0.0 : v0;
              v1 = out ? 0.0 : v1;
            }
          } else if (gy < 0 || gy >= gny) {
            v0 = 0.0;
            v1 = 0.0;
          }
          if constexpr ((ABL & 16) != 0)
            asm volatile("" ::"v"(v0), "v"(v1));  // ablation: no u^{t+1} LDS write
          else
            *reinterpret_cast<double2 *>(u1buf + uslot(m, q - 2 * E) * U1W + R * lane) = make_double2(v0, v1);
          if constexpr (TEST)
            *reinterpret_cast<double2 *>(qbuf + uslot(m, q - 2 * E) * U1W + R * lane) = make_double2(q0, q1);
        }
        if constexpr ((ABL & 4096) != 0)
          asm volatile("s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0");
        if constexpr ((ABL & 40) != 40) {
          if constexpr (RB::LEAN) {
            if constexpr ((q & (B - 1)) == B - 1) row_barrier();
          } else if ((i & (B - 1)) == B - 1) {
            row_barrier();
          }
        }
        // lean rows have no branch between them: without a scheduling fence
        // per row hipcc interleaves whole periods and spills
        if constexpr (RB::LEAN) __builtin_amdgcn_sched_barrier(0);
    };
    if constexpr (HEAD) {  // n_in >= 4E+1 >= P: every row of the first period exists
      static_for<P>([&](auto qc) __attribute__((always_inline)) {
        constexpr int q = decltype(qc)::value;
        body(qc, PairRowBounds<(q < 2 * E ? E - q : -E), E, (q + 1 < 2 * E ? E - q - 1 : -E), E>{});
      });
      bs = P & (K - 1);
      b = P;
    }
    // OPT & 128: the last X1 rows in two period-aligned parts (tail_ok: this
    // segment's n_in has the congruence pair_tail_c names)
    constexpr int TC = (OPT & 128) != 0 ? pair_tail_c(E) : -1;
    constexpr int X1 = TC >= 0 ? pair_tail_len(E, TC) : 0;
    const bool tail_ok = TC >= 0 && HEAD && n_in >= P + X1 && (n_in - TC) % P == 0;
    const int bend = tail_ok ? n_in - X1 : n_in;
    // OPT & 256: the periods after the head that lie wholly inside the
    // segment's rows run lean (past the warm-up: b >= P > 2E); the rest of
    // the rows (a partial last period) take the checked body.  Sequential
    // loops, not a lean / checked choice per period: hipcc spills when one
    // loop holds two copies of the period
    constexpr bool LEANOK = (OPT & 256) != 0 && HEAD && (P % B) == 0 && (ABL & 32) == 0;
    static_assert(!LEANOK || P >= 2 * E, "lean periods start past the warm-up");
    if constexpr (LEANOK) {
      // OPT & 4096: lean periods end before the segment's last E u^{t+1} rows
      const int lean_end = (OPT & 4096) != 0 ? min(bend, n_in - E) : bend;
      for (; b + P <= lean_end; b += P) {
        static_for<P>([&](auto qc) __attribute__((always_inline)) {
          body(qc, PairRowBounds<-E, E, -E, E, true>{});
        });
        bs = (bs + P) & (K - 1);
      }
    }
    for (; b < bend; b += P) {
      static_for<P>([&](auto qc) __attribute__((always_inline)) { body(qc, PairRowBounds<-E, E, -E, E>{}); });
      bs = (bs + P) & (K - 1);
    }
    if constexpr (TC >= 0) {
      if (tail_ok) {
        static_for<(X1 + P - 1) / P>([&](auto pc) __attribute__((always_inline)) {
          constexpr int part = decltype(pc)::value;
          static_for<P>([&](auto qc) __attribute__((always_inline)) {
            constexpr int r = part * P + decltype(qc)::value;  // tail row: i = n_in - X1 + r
            if constexpr (r < X1) body(qc, PairRowBounds<-E, X1 - 1 - r - E, -E, X1 - 2 - r - E>{});
          });
          b += P;
          bs = (bs + P) & (K - 1);
        });
      }
    }
    // the block-end barriers of wave 1's iterations n_in .. i_last
    for (int j = (i_last + 1) / B - n_in / B; j > 0; --j) row_barrier();
  } else {
    // ---- memory + stage 2 on u^{t+1} row m2 = i - 2E - B
    const int yfirst = up ? (Y1 + 2 * E - 1) : (Y0 - 2 * E);
    const double *gnext = Rc.u + (int64_t)yfirst * pitch + (x0 - 2 * E);
    const uint32_t lring = __builtin_amdgcn_readfirstlane(lds_addr(ring));
    [[maybe_unused]] int row = 0;  // next u^t row to fetch (clamped at the last one; OPT & 2: unused)
    int irow = 0;  // u^t row index of the next issue (unclamped; TEST rows follow it)
    const double *lw0p = TEST ? Rc.lw + (x0 - E - LOFF) : nullptr;
    const uint32_t llw = __builtin_amdgcn_readfirstlane(lds_addr(lwr));
    const uint32_t lsy = __builtin_amdgcn_readfirstlane(lds_addr(syr));
    // SEP: the lane's two stage-1 columns' Sx'_l and sx, for the whole segment
    [[maybe_unused]] double sxp[NLV + 1][R];
    if constexpr (SEP) {
      const int64_t ncol = pair_sep_ncol(E, C.nx);
      const double *t = C.lsx + (rgx0 + x0 - E + R * lane + 2 * E);
#pragma unroll
      for (int l = 0; l <= NLV; ++l)
#pragma unroll
        for (int c = 0; c < R; ++c) sxp[l][c] = t[l * ncol + c];
    }
    [[maybe_unused]] const uint32_t ltyr = __builtin_amdgcn_readfirstlane(lds_addr(tyr));
    // SEP: L_h[W0] of the row in ring slot `slot` from its DMA'd Ty / Z row
    // (uniform LDS reads) and the lane's Sx' (registers; the host folds c dh^2
    // into them), into the slot wave 0 reads
    auto lw_compute = [&](int slot) __attribute__((always_inline)) {
      if constexpr (SEP) {
        const double *ty = tyr + slot * LTS;
        double a[R];
#pragma unroll
        for (int c = 0; c < R; ++c) {
          a[c] = sxp[NLV][c] * ty[NLV];
#pragma unroll
          for (int l = 0; l < NLV; ++l) a[c] = fma(sxp[l][c], ty[l], a[c]);
        }
        double *dl = lwr + slot * LWW + LOFF + R * lane;
        if constexpr (LOFF == 0) {
          *reinterpret_cast<double2 *>(dl) = make_double2(a[0], a[1]);
        } else {
          dl[0] = a[0];
          dl[1] = a[1];
        }
      }
    };
    auto issue = [&](int slot) {
      if constexpr (TEST) {
        // L_h[W0] and sin(2 pi y dh) of u^{t+1} row irow - 2E (stage 1's output
        // when it reads u^t row irow)
        const int m = irow - 2 * E;
        if (!(ABL & 2) && !(ABL & 256)) {
          // SEP: the Ty / Z row of u^t row irow + B (its L_h[W0] row is
          // computed by lw_compute at wave 1's iteration irow - DT, B rows
          // ahead of wave 0: landed by then, and never in the block wave 0 holds)
          if constexpr (SEP)
            dma_chunks<LTS / 2, false, false>(C.lty + (int64_t)(rgy0 + m_row(m + B) + 2 * E) * LTS,
                                              ltyr + ((slot + B) & (K - 1)) * LTS * 8, lane);
          if constexpr ((ABL & 16384) == 0 && !SEP)  // ablation 16384: no L_h[W0] row DMA
            dma_chunks<NCHL, false, false>(lw0p + (int64_t)m_row(m) * pitch, llw + slot * LWW * 8, lane);
          dma_chunks<1, false, false>(C.syt + (sy_idx(m) & ~1), lsy + slot * 16, lane);
        }
        ++irow;
      }
      // default-policy (temporal) DMA: a strip's 2E halo columns are read
      // again by its neighbours on the same XCD (L2 hits); nt loads measured
      // 1-3% slower here (profiles/r02/pair_bench_5.jsonl); ABL 1024 = nt
      if constexpr ((ABL & 1024) != 0)
        dma_chunks<NCH>(gnext, lring + slot * RW * 8, lane);
      else if (!(ABL & 2) && !(ABL & 256))
        dma_chunks<NCH, false, false>(gnext, lring + slot * RW * 8, lane);
      if constexpr ((ABL & 32) != 0 || (OPT & 2) != 0)
        gnext += stride;  // past the last input row: the block's padding rows
      else if (++row < n_in)
        gnext += stride;
    };
    if constexpr (SEP) {  // the Ty / Z rows of u^t rows 0 .. B-1 (the issues below carry rows B ..)
#pragma unroll
      for (int r = 0; r < B; ++r)
        dma_chunks<LTS / 2, false, false>(C.lty + (int64_t)(rgy0 + m_row(r - 2 * E) + 2 * E) * LTS,
                                          ltyr + r * LTS * 8, lane);
    }
#pragma unroll
    for (int s = 0; s < DT; ++s) issue(s);
    wait_vmcnt<D * GA>();  // rows 0 .. B-1 landed (D rows may still fly)
    if constexpr (SEP)
#pragma unroll
      for (int r = 0; r < B; ++r) lw_compute(r);
    row_barrier();
    const int xo = x0 + R * lane;
    const bool emit0 = R * lane < WO && xo < rx1;
    const bool emit1 = R * lane < WO && xo + 1 < rx1;
    // OPT & 4: the lane that stores one column (an odd-width rect's last one)
    // behind a wave-uniform test, so the common row takes one masked store
    const bool single = emit0 && !emit1;
    const bool any_single = __builtin_amdgcn_ballot_w64(single) != 0;
    double *const run = Rc.un;
    const int yout0 = up ? Y1 - 1 : Y0;
    // block end at iteration j: wave 0 next reads rows j+1 .. j+B, so row
    // j+B (issued first thing in iteration j+B-DT = j-D) must have landed.
    // Issued after it: the DMAs of iterations j-D+1 .. j (D*G) and the
    // stores of iterations j-D .. j (at least one each once stores have
    // begun, iteration 4E+B; more outstanding only makes the wait longer)
    auto block_end = [&](int j) {
      if ((j & (B - 1)) != B - 1) return;
      if constexpr ((ABL & 64) != 0) {
        row_barrier();  // ablation: no wait for the DMA'd rows
        return;
      }
      if (j - D >= 4 * E + B)
        wait_vmcnt<D * GA + D + 1>();
      else
        wait_vmcnt<D * GA>();
      row_barrier();
    };
    // iterations 0 .. P-1 have no u^{t+1} row yet (m2 < 0; n_in > P always):
    // fetch + barrier only.  Peeled, so the accumulators never sit under a
    // branch (a conditional scatter makes the compiler copy them around)
    for (int i = 0; i < P; ++i) {
      issue(RP ? (i + DT < K ? i + DT : i + DT - K) : (i + DT) & (K - 1));
      lw_compute((i + B) & (K - 1));  // SEP: the L_h[W0] row of u^t row i + B
      block_end(i);
    }
    int bs = P & (K - 1);  // b % K
    // OPT & 1: output row of iteration i (row yout0 + ydir (m2 - 2E)), advanced
    // by one row per iteration; starts at i = P
    double *dstp = run + (int64_t)(yout0 + ydir * (P - 4 * E - B)) * pitch;
    int b = P;
    auto body = [&](auto qc, auto bc) __attribute__((always_inline)) {
        constexpr int q = decltype(qc)::value;
        using RB = decltype(bc);
        constexpr int LO2 = RB::LO, HI2 = RB::HI;
        constexpr int q2 = ((q - 2 * E - B) % P + P) % P;  // slot of row m2 = i - 2E - B (same parity as i)
        constexpr int so = (q2 + P - E) % P;
        const int i = b + q;
        if constexpr ((ABL & 32) == 0 && !RB::LEAN)
          if (i > i_last) return;
        issue(kslot(bs, q + DT));  // u^t row i+DT (clamped; never a slot wave 0 still reads)
        lw_compute(kslot(bs, q + B));  // SEP: the L_h[W0] row of u^t row i + B
        // u^{t+1} row m2 = i - 2E - B (m2 mod P == q2); rows m2 < 0 are LDS
        // garbage that only reaches accumulators of rows never emitted, each
        // assigned afresh before use
        const int m2 = i - 2 * E - B;
        // OPT & 32: u^{t+1} row m2+1 was written by wave 0 in the previous block
        double (&w2)[NW] = wr[q & 1];
        if constexpr (!PF || (q & 1) == 0) window(u1buf + uslot(m2, q - 2 * E - B) * U1W + R * lane, w2);
        if constexpr (PF && (q & 1) == 0) window(u1buf + uslot(m2 + 1, q + 1 - 2 * E - B) * U1W + R * lane, wr[1]);
        if constexpr (PI) {
          static_assert((q2 & 1) == (q & 1), "row pairs follow the barrier blocks");
          if constexpr ((q & 1) == 0)
            pair_levels2<E, pair_head_lmax<E, LO2, HI2>(), pair_head_lmax<E, RB::LON, RB::HIN>()>(
                wr[0], wr[1], hv[0], hv[1]);
          pair_taps<E, q2, 1 + (q2 & 1), LO2, HI2>(w2, hv[q & 1], hv[0], acc, kc);
        } else {
          pair_scatter<E, q2, PAIRS ? 1 + (q2 & 1) : 0, LO2, HI2>(w2, acc, kc, hs);
        }
        if constexpr (TEST) {  // (dt/alpha) b(t+1) at the centre row of the output
          const double *qr = qbuf + uslot(m2, q - 2 * E - B) * U1W + R * lane + E;
          acc[0][q2] += qr[0];
          acc[1][q2] += qr[1];
        }
        if (RB::LEAN || (ABL & 32) != 0 || m2 >= 2 * E) {
          const double o0 = alpha * acc[0][so];
          const double o1 = alpha * acc[1][so];
          double *dst = (OPT & 1) ? dstp : run + (int64_t)(yout0 + ydir * (m2 - 2 * E)) * pitch;
          if constexpr ((ABL & 2) != 0 || (ABL & 128) != 0) {
            asm volatile("" ::"v"(o0), "v"(o1));
          } else if constexpr ((ABL & 512) != 0) {  // ablation: non-temporal stores
            if (emit1) {
              __builtin_nontemporal_store(o0, dst + xo);
              __builtin_nontemporal_store(o1, dst + xo + 1);
            } else if (emit0) {
              __builtin_nontemporal_store(o0, dst + xo);
            }
          } else if constexpr ((OPT & 4) != 0) {
            if (emit1) *reinterpret_cast<double2 *>(dst + xo) = make_double2(o0, o1);
            if (any_single)
              if (single) dst[xo] = o0;
          } else if (emit1) {
            *reinterpret_cast<double2 *>(dst + xo) = make_double2(o0, o1);
          } else if (emit0) {
            dst[xo] = o0;
          }
        }
        if constexpr ((OPT & 1) != 0) dstp += stride;
        if constexpr ((ABL & 8192) != 0)
          asm volatile("s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0");
        if constexpr ((ABL & 40) != 40) {
          if constexpr (RB::LEAN && (ABL & 64) == 0) {
            // lean: a block end is a template constant and stores have begun
            // the stores of iterations j-D+1 .. j (D) follow row j+B's DMA
            // at every lean block end j (b >= 2P; static_assert below)
            if constexpr ((q & (B - 1)) == B - 1) {
              wait_vmcnt<D * GA + D>();
              row_barrier();
            }
          } else {
            block_end(i);
          }
        }
        if constexpr (RB::LEAN) __builtin_amdgcn_sched_barrier(0);
    };
    // head period (b == P): m2 = q + P - 2E - B, outputs m2+d < E never emitted
    constexpr auto head_lo = [](int m) constexpr { return m < 2 * E ? (E - m > E + 1 ? E + 1 : E - m) : -E; };
    if constexpr ((OPT & 16) != 0) {
      static_for<P>([&](auto qc) __attribute__((always_inline)) {
        constexpr int m2h = decltype(qc)::value + P - 2 * E - B;
        body(qc, PairRowBounds<head_lo(m2h), E, head_lo(m2h + 1), E>{});
      });
      bs = (bs + P) & (K - 1);
      b += P;
    }
    // OPT & 128: the last X2 iterations, outputs m2+d >= nm - E never emitted
    constexpr int TC = (OPT & 128) != 0 ? pair_tail_c(E) : -1;
    constexpr int X2 = TC >= 0 ? pair_tail_len(E, TC + B) : 0;
    const bool tail_ok = TC >= 0 && (OPT & 16) != 0 && i_last + 1 - X2 >= 2 * P && (n_in - TC) % P == 0;
    const int bend = tail_ok ? i_last + 1 - X2 : i_last + 1;
    // OPT & 256: the periods from the first after the head (b = 2P) that lie
    // wholly inside the iterations run lean; a partial last period the
    // checked body (sequential loops, as stage 1)
    constexpr bool LEANOK = (OPT & 1024) != 0 && (OPT & 16) != 0 && (P % B) == 0 && (ABL & 32) == 0;
    // b >= 2P: every row emits (m2 = i - 2E - B >= 2E) and at every block end
    // j the stores of iterations j-D+1 .. j have been issued (j-D+1 >= 4E+B)
    static_assert(!LEANOK || (2 * P - 2 * E - B >= 2 * E && 2 * P + B - D >= 4 * E + B), "lean from b = 2P");
    if constexpr (LEANOK) {
      // OPT & 4096: lean periods end before the segment's last E u^{t+1} rows
      const int lean_end = (OPT & 4096) != 0 ? min(bend, n_in - E) : bend;
      for (; b + P <= lean_end; b += P) {
        static_for<P>([&](auto qc) __attribute__((always_inline)) {
          body(qc, PairRowBounds<-E, E, -E, E, true>{});
        });
        bs = (bs + P) & (K - 1);
      }
    }
    for (; b < bend; b += P) {
      static_for<P>([&](auto qc) __attribute__((always_inline)) { body(qc, PairRowBounds<-E, E, -E, E>{}); });
      bs = (bs + P) & (K - 1);
    }
    if constexpr (TC >= 0) {
      if (tail_ok) {
        static_for<(X2 + P - 1) / P>([&](auto pc) __attribute__((always_inline)) {
          constexpr int part = decltype(pc)::value;
          static_for<P>([&](auto qc) __attribute__((always_inline)) {
            constexpr int r = part * P + decltype(qc)::value;  // tail iteration: i = i_last + 1 - X2 + r
            if constexpr (r < X2) body(qc, PairRowBounds<-E, X2 - 1 - r - E, -E, X2 - 2 - r - E>{});
          });
          b += P;
          bs = (bs + P) & (K - 1);
        });
      }
    }
    wait_vmcnt<0>();  // drain the tail DMAs and the stores
  }
  if constexpr ((ABL & 2048) != 0) {
    const uint64_t t_exit = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      uint64_t *rec = reinterpret_cast<uint64_t *>(const_cast<double *>(Rc.lw)) + 4 * (2 * blockIdx.x + wave);
      rec[0] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
      rec[1] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
      rec[2] = t_entry;
      rec[3] = t_exit;
    }
  }
}

// pass variants libnlh launches (the host picks one per solver):
//   6 production, 8-slot rings (D = 4, B = 2)    -- default
//   1 production, 16-slot rings (D = 8, B = 4)   -- NLH_PAIR_SPLIT=1 (tuning)
//   5 test mode, 8-slot rings (D = 4, B = 2)     -- default in test mode
//   4 test mode, 16-slot rings (D = 8, B = 4)    -- NLH_PAIR_TEST=0 (tuning)
// All four are the same arithmetic in the same order (bitwise equal fields).
// kPairNoPrio | 6 or | 5: the same kernel without the wave priority (OPT bit
// 8), which the host launches when a list has more workgroups than the device
// holds at once: with several rounds of workgroups the priority costs 1-4%
// (C2 harness 16384^2 / 32768^2: 982-991 vs 995-998 / 3861-3871 vs 4016-4027
// us per pass), in one round it gains 4% (4096^2 / 8192^2; profiles/r04/prio/).
// The no-priority launch also drops the period-aligned rings (2048) and the
// tail skip (128): with several rounds they cost 4-5% (harness OPT 6615 vs
// 4439, 16384^2: 1022-1024 vs 979-982, 32768^2: 3998-4009 vs 3794 us per
// pass; profiles/r05/pair/big*.jsonl); the lattice-edge select stays.
// Resident workgroups per CU (register/LDS-limited) for the host's choice of
// segment height; 0 for an unknown variant
template <int E>
int pair_blocks_per_cu_e(int variant) {
  int n = 0;
  hipError_t e = hipErrorInvalidValue;
  // the priority variant's residency: the host launches a list with the
  // priority only when all its workgroups are resident at once in THAT
  // variant (the no-priority one, without the period-aligned rings, holds
  // less LDS and may fit more per CU; that count decides nothing)
  variant &= ~kPairNoPrio;
  if (variant == 1) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_pair_split<E, kPairSplitD>, 128, 0);
  else if (variant == 6) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_pair_split<E, 4, 0, 2>, 128, 0);
  else if (variant == 5)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_pair_split<E, 4, 0, 2, true>, 128, 0);
  else if (variant == 4)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_pair_split<E, kPairSplitD, 0, kPairSplitB, true>, 128, 0);
  return e == hipSuccess ? n : 0;
}

template <int E>
int launch_pair_e(const RectList &rl, const StepConst &c, int variant, hipStream_t st) {
  constexpr int NP = pair_opt(E) & ~(8 | 128 | 2048);
  if (variant == 1)
    hipLaunchKernelGGL((k_pair_split<E, kPairSplitD>), dim3(rl.nwork), dim3(128), 0, st, rl, c);
  else if (variant == 6)
    hipLaunchKernelGGL((k_pair_split<E, 4, 0, 2>), dim3(rl.nwork), dim3(128), 0, st, rl, c);
  else if (variant == (kPairNoPrio | 6))
    hipLaunchKernelGGL((k_pair_split<E, 4, 0, 2, false, NP>), dim3(rl.nwork), dim3(128), 0, st, rl, c);
  else if (variant == 5)
    hipLaunchKernelGGL((k_pair_split<E, 4, 0, 2, true>), dim3(rl.nwork), dim3(128), 0, st, rl, c);
  else if (variant == (kPairNoPrio | 5))
    hipLaunchKernelGGL((k_pair_split<E, 4, 0, 2, true, NP>), dim3(rl.nwork), dim3(128), 0, st, rl, c);
  else if (variant == 4)
    hipLaunchKernelGGL((k_pair_split<E, kPairSplitD, 0, kPairSplitB, true>), dim3(rl.nwork), dim3(128), 0, st,
                       rl, c);
  else
    return (int)hipErrorInvalidValue;
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace nlh
