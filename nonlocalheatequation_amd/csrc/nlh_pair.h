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
constexpr int kPairPadRows = 16;
__host__ __device__ constexpr int pair_opt(int E) { return E == 13 ? 14 : 15; }

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
template <int E, int QA, int ROLE>
__device__ __forceinline__ void pair_scatter(const double (&w)[2 * E + 2], double (&acc)[2][pair_slots(E)],
                                             double kc, double (&hs)[2][E + 1]) {
  constexpr int P = pair_slots(E);
  constexpr int SF = (QA + E) % P;      // d = +E: first term of that output row
  constexpr int SL = (QA + P - E) % P;  // d = -E: last term
  acc[0][SF] = w[E];
  acc[1][SF] = w[E + 1];
  acc[0][SL] += w[E];
  acc[1][SL] += w[E + 1];
  // levels and taps are template constants (static_for): evaluating the
  // disk shape inside the row loop at run time costs more than the sums
  double core = w[E] + w[E + 1];
  auto level = [&](auto lc) {
    constexpr int Lv = decltype(lc)::value + 1;
    if constexpr (Lv > 1) core = core + (w[E + 1 - Lv] + w[E + Lv]);
    if constexpr (pair_level_used(E, Lv)) {
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
        if constexpr (clen(E, pair_abs(d)) == Lv) {
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
  acc[0][QA] = fma(kc, w[E], acc[0][QA]);
  acc[1][QA] = fma(kc, w[E + 1], acc[1][QA]);
}

// ABL: timing-decomposition masks for the tools/ harness (tools/pair_bench.hip).
// libnlh instantiates ABL = 0 only (tests/test_capi.py checks the library's
// kernel symbols); with ABL != 0 the results are meaningless.  k_pair_split:
// 2 = no HBM traffic (no DMA, no stores; same instruction stream otherwise),
// 4 = windows from registers (no LDS window reads), 8 = no s_barrier,
// 16 = no u^{t+1} LDS writes, 32 = no per-row range checks (rows past the
// segment end computed too), 64 = no vmcnt waits for the DMA'd rows, 128 = no
// output stores, 256 = no DMA, 512 = non-temporal stores, 1024 = non-temporal DMA

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
  constexpr int K = pow2_ceil(DT + B);  // rows i .. i+DT+B-1 live at once
  constexpr int G = (NCH + 63) / 64;
  constexpr int U1W = W1 + 2 * E + 2;
  constexpr int U1R = 2 * B;            // u^{t+1} ring rows
  // TEST: L_h[W0] row of the stage-1 columns x0-E .. x0-E+W1-1, staged from
  // the even column at or before x0-E (16-byte DMA chunks)
  constexpr int LOFF = E & 1;
  constexpr int NCHL = TEST ? (W1 + LOFF + 1) / 2 : 0;
  constexpr int LWW = 2 * NCHL;
  constexpr int GT = TEST ? (NCHL + 63) / 64 + 1 : 0;  // + the sin(2 pi y dh) pair
  constexpr int GA = G + GT;            // DMA instructions per row
  static_assert((B & (B - 1)) == 0, "B must be a power of two");
  static_assert(D * GA + D + 1 < 64, "vmcnt range");
  static_assert(WO >= 64, "strip too narrow for this eps");
  static_assert(P <= 2 * E + B, "the peeled iterations 0 .. P-1 carry no u^{t+1} row");
  static_assert((OPT & 2) == 0 || 2 * B + D <= kPairPadRows, "tail DMAs past the padding rows");

  __shared__ __attribute__((aligned(16))) double ring[K * RW + U1R * U1W + (TEST ? U1R * U1W + K * LWW + 2 * K : 0)];
  double *const u1buf = ring + K * RW;
  double *const qbuf = u1buf + U1R * U1W;  // TEST: (dt/alpha) b(t+1) of the u^{t+1} rows
  double *const lwr = qbuf + U1R * U1W;    // TEST: L_h[W0] rows, slots of the u^t ring
  double *const syr = lwr + K * LWW;       // TEST: sin(2 pi y dh) pairs, same slots

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

  // barriers: one prologue barrier, then one after every iteration i with
  // i % B == B-1, for i = 0 .. i_last (wave 0 stops computing at n_in - 1)
  if constexpr ((OPT & 8) != 0)
    if (wave == 1) __builtin_amdgcn_s_setprio(3);
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
    for (int b = 0; b < n_in; b += P) {
      auto body = [&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int so = (q + P - E) % P;  // output row i - E completes
        const int i = b + q;
        if constexpr ((ABL & 32) == 0)
          if (i >= n_in) return;
        double w[NW];
        window(ring + ((bs + q) & (K - 1)) * RW + R * lane, w);
        pair_scatter<E, q, PAIRS ? 1 + (q & 1) : 0>(w, acc, kc, hs);
        if ((ABL & 32) != 0 || i >= 2 * E) {
          const int m = i - 2 * E;
          const int gy = gy1first + ydir * m;
          double v0 = mcol[0] * acc[0][so];
          double v1 = mcol[1] * acc[1][so];
          double q0 = 0.0, q1 = 0.0;
          if constexpr (TEST) {
            const int slot = (bs + q) & (K - 1);  // u^t row i: its L_h[W0] / sin rows
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
          if (gy < 0 || gy >= gny) {
            v0 = 0.0;
            v1 = 0.0;
          }
          if constexpr ((ABL & 16) != 0)
            asm volatile("" ::"v"(v0), "v"(v1));  // ablation: no u^{t+1} LDS write
          else
            *reinterpret_cast<double2 *>(u1buf + (m & (U1R - 1)) * U1W + R * lane) = make_double2(v0, v1);
          if constexpr (TEST)
            *reinterpret_cast<double2 *>(qbuf + (m & (U1R - 1)) * U1W + R * lane) = make_double2(q0, q1);
        }
        if constexpr ((ABL & 40) != 40)
          if ((i & (B - 1)) == B - 1) row_barrier();
      };
      static_for<P>(body);
      bs = (bs + P) & (K - 1);
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
    auto issue = [&](int slot) {
      if constexpr (TEST) {
        // L_h[W0] and sin(2 pi y dh) of u^{t+1} row irow - 2E (stage 1's output
        // when it reads u^t row irow)
        const int m = irow - 2 * E;
        if (!(ABL & 2) && !(ABL & 256)) {
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
#pragma unroll
    for (int s = 0; s < DT; ++s) issue(s);
    wait_vmcnt<D * GA>();  // rows 0 .. B-1 landed (D rows may still fly)
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
      issue((i + DT) & (K - 1));
      block_end(i);
    }
    int bs = P & (K - 1);  // b % K
    // OPT & 1: output row of iteration i (row yout0 + ydir (m2 - 2E)), advanced
    // by one row per iteration; starts at i = P
    double *dstp = run + (int64_t)(yout0 + ydir * (P - 4 * E - B)) * pitch;
    for (int b = P; b <= i_last; b += P) {
      auto body = [&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int q2 = ((q - 2 * E - B) % P + P) % P;  // slot of row m2 = i - 2E - B (same parity as i)
        constexpr int so = (q2 + P - E) % P;
        const int i = b + q;
        if constexpr ((ABL & 32) == 0)
          if (i > i_last) return;
        issue((bs + q + DT) & (K - 1));  // u^t row i+DT (clamped; never a slot wave 0 still reads)
        // u^{t+1} row m2 = i - 2E - B (m2 mod P == q2); rows m2 < 0 are LDS
        // garbage that only reaches accumulators of rows never emitted, each
        // assigned afresh before use
        const int m2 = i - 2 * E - B;
        double w2[NW];
        window(u1buf + (m2 & (U1R - 1)) * U1W + R * lane, w2);
        pair_scatter<E, q2, PAIRS ? 1 + (q2 & 1) : 0>(w2, acc, kc, hs);
        if constexpr (TEST) {  // (dt/alpha) b(t+1) at the centre row of the output
          const double *qr = qbuf + (m2 & (U1R - 1)) * U1W + R * lane + E;
          acc[0][q2] += qr[0];
          acc[1][q2] += qr[1];
        }
        if ((ABL & 32) != 0 || m2 >= 2 * E) {
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
        if constexpr ((ABL & 40) != 40) block_end(i);
      };
      static_for<P>(body);
      bs = (bs + P) & (K - 1);
    }
    wait_vmcnt<0>();  // drain the tail DMAs and the stores
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
// us per pass), in one round it gains 4% (4096^2 / 8192^2; profiles/r04/prio/)
// Resident workgroups per CU (register/LDS-limited) for the host's choice of
// segment height; 0 for an unknown variant
template <int E>
int pair_blocks_per_cu_e(int variant) {
  int n = 0;
  hipError_t e = hipErrorInvalidValue;
  variant &= ~kPairNoPrio;  // same resources with or without the priority
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
  constexpr int NP = pair_opt(E) & ~8;
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
