// pair_variants.h -- alternate two-step pass designs kept for the timing
// harness (tools/pair_bench.hip) only; libnlh ships k_pair_split
// (nonlocalheatequation_amd/csrc/nlh_pair.h).  All three are bitwise equal to the round-3
// k_pair_split; DESIGN.md section 4 records why k_pair_split won.
//   k_pair     one wave runs both stages (two accumulator sets per lane)
//   k_pair_pf  k_pair_split with the next row's LDS window read ahead
//   k_pair_mw  k_pair_split plus a third wave for all HBM traffic
#pragma once

#include "pair_split_r3.h"

namespace nlh {

constexpr int kPairD = 7;    // k_pair: u^t rows in flight per wave (ring of 8 slots)
constexpr int kPairMwD = 6;  // k_pair_mw: rows in flight beyond the next block

// ABL masks as k_pair_split's (nlh_pair.h)
template <int E, int D, int ABL = 0>
__global__ __launch_bounds__(64, (E <= 9 ? 2 : 1)) void k_pair(RectList L, StepConst C) {
  constexpr int R = 2;
  constexpr int P = 2 * E + 1;
  constexpr int W1 = 64 * R;          // u^{t+1} columns per strip
  constexpr int WO = W1 - 2 * E;      // output columns per strip
  constexpr int NW = R + 2 * E;       // window values per lane
  constexpr int RW = W1 + 2 * E;      // staged u^t doubles per ring row
  constexpr int NCH = RW / 2;         // 16-byte chunks per row
  constexpr int K = pow2_ceil(D + 1); // ring slots
  constexpr int G = (NCH + 63) / 64;  // DMA instructions per row
  constexpr int U1W = W1 + 2 * E + 2; // u^{t+1} row + read-over pad (lanes >= WO/R)
  // read the u^t window before the stage-2 math where both windows and the
  // 2 x 2(2E+1) accumulators still fit the 256 registers of two waves per
  // SIMD without spilling (hipcc 7.2 register counts: E = 7 spills with the
  // early read, E >= 9 spill either way)
  constexpr bool EARLY = E <= 6 || E == 8;
  // stores count in vmcnt (see k_fast); lane 0 always owns an output column
  static_assert(D * G + D < 64, "vmcnt range");
  static_assert(K > D, "ring slots");
  static_assert(WO >= 64, "strip too narrow for this eps");

  __shared__ __attribute__((aligned(16))) double ring[K * RW + 2 * U1W];
  double *const u1buf = ring + K * RW;

  const int lane = (int)threadIdx.x;
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  const Rect &Rc = L.r[ri];
  const double *const ru = Rc.u;
  double *const run = Rc.un;
  const int rx1 = Rc.x1, rgx0 = Rc.gx0, rgy0 = Rc.gy0;
  const int local = work - Rc.wg_begin;
  const int nstrip = Rc.nstrip;
  const int strip = local % nstrip, seg = local / nstrip;
  const int x0 = Rc.x0 + strip * WO;
  const int seg_h = Rc.seg_rows;
  const int Y0 = Rc.y0 + seg * seg_h;
  const int Y1 = min(Y0 + seg_h, Rc.y1);
  const int n_in = (Y1 - Y0) + 4 * E;   // u^t rows Y0-2E .. Y1+2E-1
  const bool up = (seg & 1) != 0;       // alternating sweep direction
  const int64_t pitch = Rc.pitch;
  const int64_t stride = up ? -pitch : pitch;
  const int yfirst = up ? (Y1 + 2 * E - 1) : (Y0 - 2 * E);
  const double alpha = C.alpha, kc = C.kc;
  const int gny = (int)C.ny;
  // u^{t+1} row m is block-local row y1first + ydir*m; global row rgy0 + that
  const int gy1first = rgy0 + (up ? (Y1 + E - 1) : (Y0 - E));
  const int ydir = up ? -1 : 1;
  const int yout0 = up ? Y1 - 1 : Y0;   // block row of the first output row

  // lane constants: alpha on the u^{t+1} columns inside the lattice, 0 outside
  double mcol[R];
#pragma unroll
  for (int c = 0; c < R; ++c) {
    const int gx = rgx0 + x0 - E + R * lane + c;
    mcol[c] = (gx >= 0 && gx < (int)C.nx) ? alpha : 0.0;
  }
  const int xo = x0 + R * lane;  // first output column of this lane
  const bool emit0 = R * lane < WO && xo < rx1;
  const bool emit1 = R * lane < WO && xo + 1 < rx1;

  const double *gnext = ru + (int64_t)yfirst * pitch + (x0 - 2 * E);
  const uint32_t lring = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  auto issue = [&](int i, int slot) {
    if (!(ABL & 2)) dma_chunks<NCH>(gnext, lring + slot * RW * 8, lane);
    if (i + 1 < n_in) gnext += stride;
  };
#pragma unroll
  for (int s = 0; s < D; ++s) issue(s, s);

  double acc1[R][P], acc2[R][P];
#pragma unroll
  for (int c = 0; c < R; ++c)
#pragma unroll
    for (int j = 0; j < P; ++j) {
      acc1[c][j] = 0.0;
      acc2[c][j] = 0.0;
    }

  // iterations i = 0 .. n_in: stage 1 on u^t row i (i = n_in re-reads the
  // clamped last row, its result is never used), stage 2 on u^{t+1} row
  // i-2E-1 (rows < 0 are LDS garbage that only reaches accumulators of rows
  // that are never emitted and are assigned afresh before use)
  int bs = 0;  // b % K
  for (int b = 0; b <= n_in; b += P) {
    // static unroll over the accumulator period: every slot index below is a
    // compile-time constant, so acc1/acc2 stay in registers
    auto body = [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      constexpr int so = (q + E + 1) % P;  // slot whose row is complete now
      const int i = b + q;
      if (i > n_in) return;
      // one row per scheduling region: letting the scheduler mix unrolled
      // rows lengthens live ranges past the 256-register budget at some E
      __builtin_amdgcn_sched_barrier(0);
      const int slot = (bs + q) & (K - 1);
      issue(i + D, (bs + q + D) & (K - 1));
      if (i >= 4 * E + 1 + D)
        wait_vmcnt<D * G + D>();
      else
        wait_vmcnt<D * G>();

      const int m2 = i - P;  // u^{t+1} row of stage 2; m2 mod P == q
      double w2[NW], w[NW];
      pair_window<E, R>(u1buf + (m2 & 1) * U1W + R * lane, w2);
      if constexpr (EARLY) pair_window<E, R>(ring + slot * RW + R * lane, w);

      // stage 2: u^{t+1} row m2 -> u^{t+2} row m2 - E complete
      pair_scatter_r3<E, q>(w2, acc2, kc);
      if (m2 >= 2 * E) {
        const double o0 = alpha * acc2[0][so];
        const double o1 = alpha * acc2[1][so];
        double *dst = run + (int64_t)(yout0 + ydir * (m2 - 2 * E)) * pitch;
        if constexpr ((ABL & 2) != 0) {
          asm volatile("" ::"v"(o0), "v"(o1));
        } else if (emit1) {
          *reinterpret_cast<double2 *>(dst + xo) = make_double2(o0, o1);
        } else if (emit0) {
          dst[xo] = o0;
        }
      }

      // stage 1: u^t row i -> u^{t+1} row m = i - 2E complete
      if constexpr (!EARLY) pair_window<E, R>(ring + slot * RW + R * lane, w);
      pair_scatter_r3<E, q>(w, acc1, kc);
      if (i >= 2 * E) {
        const int m = i - 2 * E;
        const int gy = gy1first + ydir * m;
        double v0 = mcol[0] * acc1[0][so];
        double v1 = mcol[1] * acc1[1][so];
        if (gy < 0 || gy >= gny) {
          v0 = 0.0;
          v1 = 0.0;
        }
        asm volatile("" ::: "memory");  // earlier window reads stay before this write
        *reinterpret_cast<double2 *>(u1buf + (m & 1) * U1W + R * lane) = make_double2(v0, v1);
        asm volatile("" ::: "memory");  // LDS is in order per wave: the next reads see every lane's write
      }
    };
    static_for<P>(body);
    bs = (bs + P) & (K - 1);
  }
  wait_vmcnt<0>();  // drain the clamped tail DMAs before the wave retires
}

// window buffer of row q of an unroll period of P rows: consecutive rows, the
// wrap P-1 -> 0 included, never share one (three buffers for odd P)
template <int P>
__host__ __device__ constexpr int pf_slot(int q) {
  return (P % 2 == 1 && q == P - 1) ? 2 : (q & 1);
}

// k_pair_pf: k_pair_split with the LDS window of the NEXT row read before the
// math of the current one (software pipelining), so the ds_read latency of a
// row hides behind the previous row's adds instead of stalling every row.
// Row i+1 is prefetched unless row i ends a barrier block (its data is only
// guaranteed after the barrier: then it is read right after it).  Same
// arithmetic and order as k_pair_split: bitwise equal results.
template <int E, int D, int ABL = 0, int B = kPairSplitB>
__global__ __launch_bounds__(128, 2) void k_pair_pf(RectList L, StepConst C) {
  constexpr int R = 2;
  constexpr int P = 2 * E + 1;
  constexpr int W1 = 64 * R;
  constexpr int WO = W1 - 2 * E;
  constexpr int NW = R + 2 * E;
  constexpr int RW = W1 + 2 * E;
  constexpr int NCH = RW / 2;
  constexpr int DT = B + D;
  constexpr int K = pow2_ceil(DT + B);
  constexpr int G = (NCH + 63) / 64;
  constexpr int U1W = W1 + 2 * E + 2;
  constexpr int U1R = 2 * B;
  static_assert((B & (B - 1)) == 0, "B must be a power of two");
  static_assert(D * G + D + 1 < 64, "vmcnt range");
  static_assert(WO >= 64, "strip too narrow for this eps");

  __shared__ __attribute__((aligned(16))) double ring[K * RW + U1R * U1W];
  double *const u1buf = ring + K * RW;

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
  const int n_in = (Y1 - Y0) + 4 * E;
  const int i_last = n_in - 1 + B;
  const bool up = (seg & 1) != 0;
  const int64_t pitch = Rc.pitch;
  const int64_t stride = up ? -pitch : pitch;
  const double alpha = C.alpha, kc = C.kc;
  const int ydir = up ? -1 : 1;

  auto row_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  double acc[R][P];
#pragma unroll
  for (int c = 0; c < R; ++c)
#pragma unroll
    for (int j = 0; j < P; ++j) acc[c][j] = 0.0;
  double wb[3][NW];  // window buffers (pf_slot); SSA values after unrolling

  if (wave == 0) {
    // ---- stage 1 on u^t row i
    const int gny = (int)C.ny;
    const int gy1first = rgy0 + (up ? (Y1 + E - 1) : (Y0 - E));
    double mcol[R];
#pragma unroll
    for (int c = 0; c < R; ++c) {
      const int gx = rgx0 + x0 - E + R * lane + c;
      mcol[c] = (gx >= 0 && gx < (int)C.nx) ? alpha : 0.0;
    }
    auto ring_row = [&](int r) { return ring + (r & (K - 1)) * RW + R * lane; };
    row_barrier();  // prologue: rows 0 .. B-1 landed
    pair_window<E, R>(ring_row(0), wb[0]);
    int bs = 0;     // b % K
    for (int b = 0; b < n_in; b += P) {
      auto body = [&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int so = (q + E + 1) % P;
        constexpr int cs = pf_slot<P>(q), ns = pf_slot<P>((q + 1) % P);
        const int i = b + q;
        if (i >= n_in) return;
        const bool bend = (i & (B - 1)) == B - 1;
        const bool more = i + 1 < n_in;
        if (more && !bend) pair_window<E, R>(ring_row(bs + q + 1), wb[ns]);
        pair_scatter_r3<E, q>(wb[cs], acc, kc);
        if (i >= 2 * E) {
          const int m = i - 2 * E;
          const int gy = gy1first + ydir * m;
          double v0 = mcol[0] * acc[0][so];
          double v1 = mcol[1] * acc[1][so];
          if (gy < 0 || gy >= gny) {
            v0 = 0.0;
            v1 = 0.0;
          }
          *reinterpret_cast<double2 *>(u1buf + (m & (U1R - 1)) * U1W + R * lane) = make_double2(v0, v1);
        }
        if (bend) {
          row_barrier();
          if (more) pair_window<E, R>(ring_row(bs + q + 1), wb[ns]);
        }
      };
      static_for<P>(body);
      bs = (bs + P) & (K - 1);
    }
    for (int j = (i_last + 1) / B - n_in / B; j > 0; --j) row_barrier();
  } else {
    // ---- memory + stage 2 on u^{t+1} row m2 = i - 2E - B
    const int yfirst = up ? (Y1 + 2 * E - 1) : (Y0 - 2 * E);
    const double *gnext = Rc.u + (int64_t)yfirst * pitch + (x0 - 2 * E);
    const uint32_t lring = __builtin_amdgcn_readfirstlane(lds_addr(ring));
    int row = 0;
    auto issue = [&](int slot) {
      if (!(ABL & 2)) dma_chunks<NCH>(gnext, lring + slot * RW * 8, lane);
      if (++row < n_in) gnext += stride;
    };
#pragma unroll
    for (int s = 0; s < DT; ++s) issue(s);
    wait_vmcnt<D * G>();
    row_barrier();
    const int xo = x0 + R * lane;
    const bool emit0 = R * lane < WO && xo < rx1;
    const bool emit1 = R * lane < WO && xo + 1 < rx1;
    double *const run = Rc.un;
    const int yout0 = up ? Y1 - 1 : Y0;
    auto u1_row = [&](int m) { return u1buf + (m & (U1R - 1)) * U1W + R * lane; };
    auto block_end = [&](int j) {
      if ((j & (B - 1)) != B - 1) return;
      if (j - D >= 4 * E + B)
        wait_vmcnt<D * G + D + 1>();
      else
        wait_vmcnt<D * G>();
      row_barrier();
    };
    for (int i = 0; i < P; ++i) {
      issue((i + DT) & (K - 1));
      block_end(i);
    }
    pair_window<E, R>(u1_row(P - 2 * E - B), wb[0]);  // the first main iteration's row
    int bs = P & (K - 1);
    for (int b = P; b <= i_last; b += P) {
      auto body = [&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int q2 = ((q + 1 - B) % P + P) % P;
        constexpr int so = (q2 + E + 1) % P;
        constexpr int cs = pf_slot<P>(q), ns = pf_slot<P>((q + 1) % P);
        const int i = b + q;
        if (i > i_last) return;
        issue((bs + q + DT) & (K - 1));
        const int m2 = i - 2 * E - B;
        const bool bend = (i & (B - 1)) == B - 1;
        const bool more = i + 1 <= i_last;
        if (more && !bend) pair_window<E, R>(u1_row(m2 + 1), wb[ns]);
        pair_scatter_r3<E, q2>(wb[cs], acc, kc);
        if (m2 >= 2 * E) {
          const double o0 = alpha * acc[0][so];
          const double o1 = alpha * acc[1][so];
          double *dst = run + (int64_t)(yout0 + ydir * (m2 - 2 * E)) * pitch;
          if constexpr ((ABL & 2) != 0) {
            asm volatile("" ::"v"(o0), "v"(o1));
          } else if (emit1) {
            *reinterpret_cast<double2 *>(dst + xo) = make_double2(o0, o1);
          } else if (emit0) {
            dst[xo] = o0;
          }
        }
        if (bend) {
          block_end(i);
          if (more) pair_window<E, R>(u1_row(m2 + 1), wb[ns]);
        }
      };
      static_for<P>(body);
      bs = (bs + P) & (K - 1);
    }
    wait_vmcnt<0>();
  }
}

// k_pair_mw: k_pair_split with all HBM traffic on a third wave, so the two
// arithmetic waves never issue a global memory instruction:
//   wave 0: stage 1 (as k_pair_split);
//   wave 1: stage 2, u^{t+2} rows into a 2B-row LDS output ring;
//   wave 2: LDS-DMA of u^t rows (and the block-end waits), and the copy of
//           each finished u^{t+2} row LDS -> HBM one block after wave 1 wrote
//           it.
// Barriers at every block end of iterations 0 .. n_in-1+2B (+ one prologue
// barrier), all three waves.  Bitwise equal to k_pair_split.
template <int E, int D, int ABL = 0, int B = 2>
__global__ __launch_bounds__(192, 3) void k_pair_mw(RectList L, StepConst C) {
  constexpr int R = 2;
  constexpr int P = 2 * E + 1;
  constexpr int W1 = 64 * R;
  constexpr int WO = W1 - 2 * E;
  constexpr int NW = R + 2 * E;
  constexpr int RW = W1 + 2 * E;
  constexpr int NCH = RW / 2;
  constexpr int DT = B + D;
  constexpr int K = pow2_ceil(DT + B);
  constexpr int G = (NCH + 63) / 64;
  constexpr int U1W = W1 + 2 * E + 2;
  constexpr int U1R = 2 * B;
  static_assert((B & (B - 1)) == 0, "B must be a power of two");
  static_assert(D * G + D + 1 < 64, "vmcnt range");
  static_assert(WO >= 64, "strip too narrow for this eps");

  __shared__ __attribute__((aligned(16))) double ring[K * RW + U1R * U1W + U1R * W1];
  double *const u1buf = ring + K * RW;
  double *const obuf = u1buf + U1R * U1W;

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
  const int n_in = (Y1 - Y0) + 4 * E;
  const int i_last = n_in - 1 + B;      // wave 1's last iteration
  const int i_end = i_last + B;         // wave 2's last iteration
  const int nbar = (i_end + 1) / B;     // block-end barriers of iterations 0 .. i_end
  const bool up = (seg & 1) != 0;
  const int64_t pitch = Rc.pitch;
  const int64_t stride = up ? -pitch : pitch;
  const double alpha = C.alpha, kc = C.kc;
  const int ydir = up ? -1 : 1;

  auto row_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  if (wave == 0) {
    // ---- stage 1 on u^t row i (as k_pair_split)
    double acc[R][P];
#pragma unroll
    for (int c = 0; c < R; ++c)
#pragma unroll
      for (int j = 0; j < P; ++j) acc[c][j] = 0.0;
    const int gny = (int)C.ny;
    const int gy1first = rgy0 + (up ? (Y1 + E - 1) : (Y0 - E));
    double mcol[R];
#pragma unroll
    for (int c = 0; c < R; ++c) {
      const int gx = rgx0 + x0 - E + R * lane + c;
      mcol[c] = (gx >= 0 && gx < (int)C.nx) ? alpha : 0.0;
    }
    row_barrier();
    int bs = 0;
    for (int b = 0; b < n_in; b += P) {
      auto body = [&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int so = (q + E + 1) % P;
        const int i = b + q;
        if (i >= n_in) return;
        double w[NW];
        pair_window<E, R>(ring + ((bs + q) & (K - 1)) * RW + R * lane, w);
        pair_scatter_r3<E, q>(w, acc, kc);
        if (i >= 2 * E) {
          const int m = i - 2 * E;
          const int gy = gy1first + ydir * m;
          double v0 = mcol[0] * acc[0][so];
          double v1 = mcol[1] * acc[1][so];
          if (gy < 0 || gy >= gny) {
            v0 = 0.0;
            v1 = 0.0;
          }
          *reinterpret_cast<double2 *>(u1buf + (m & (U1R - 1)) * U1W + R * lane) = make_double2(v0, v1);
        }
        if ((i & (B - 1)) == B - 1) row_barrier();
      };
      static_for<P>(body);
      bs = (bs + P) & (K - 1);
    }
    for (int j = nbar - n_in / B; j > 0; --j) row_barrier();
  } else if (wave == 1) {
    // ---- stage 2 on u^{t+1} row m2 = i - 2E - B; u^{t+2} row k = m2 - 2E
    // into the output ring
    double acc[R][P];
#pragma unroll
    for (int c = 0; c < R; ++c)
#pragma unroll
      for (int j = 0; j < P; ++j) acc[c][j] = 0.0;
    row_barrier();
    for (int i = 0; i < P; ++i)
      if ((i & (B - 1)) == B - 1) row_barrier();
    for (int b = P; b <= i_last; b += P) {
      auto body = [&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int q2 = ((q + 1 - B) % P + P) % P;
        constexpr int so = (q2 + E + 1) % P;
        const int i = b + q;
        if (i > i_last) return;
        const int m2 = i - 2 * E - B;
        double w2[NW];
        pair_window<E, R>(u1buf + (m2 & (U1R - 1)) * U1W + R * lane, w2);
        pair_scatter_r3<E, q2>(w2, acc, kc);
        if (m2 >= 2 * E) {
          const int k = m2 - 2 * E;
          *reinterpret_cast<double2 *>(obuf + (k & (U1R - 1)) * W1 + R * lane) =
              make_double2(alpha * acc[0][so], alpha * acc[1][so]);
        }
        if ((i & (B - 1)) == B - 1) row_barrier();
      };
      static_for<P>(body);
    }
    for (int j = nbar - (i_last + 1) / B; j > 0; --j) row_barrier();
  } else {
    // ---- memory: u^t rows in, u^{t+2} rows out
    const int yfirst = up ? (Y1 + 2 * E - 1) : (Y0 - 2 * E);
    const double *gnext = Rc.u + (int64_t)yfirst * pitch + (x0 - 2 * E);
    const uint32_t lring = __builtin_amdgcn_readfirstlane(lds_addr(ring));
    int row = 0;
    auto issue = [&](int slot) {
      if (!(ABL & 2)) dma_chunks<NCH>(gnext, lring + slot * RW * 8, lane);
      if (++row < n_in) gnext += stride;
    };
#pragma unroll
    for (int s = 0; s < DT; ++s) issue(s);
    wait_vmcnt<D * G>();
    row_barrier();
    const int xo = x0 + R * lane;
    const bool emit0 = R * lane < WO && xo < rx1;
    const bool emit1 = R * lane < WO && xo + 1 < rx1;
    double *const run = Rc.un;
    const int yout0 = up ? Y1 - 1 : Y0;
    const int nout = Y1 - Y0;
    for (int i = 0; i <= i_end; ++i) {
      issue((i + DT) & (K - 1));
      // u^{t+2} row k finished by wave 1 one block ago
      const int k = i - 4 * E - 2 * B;
      if (k >= 0 && k < nout) {
        const double2 o = *reinterpret_cast<const double2 *>(obuf + (k & (U1R - 1)) * W1 + R * lane);
        double *dst = run + (int64_t)(yout0 + ydir * k) * pitch;
        if constexpr ((ABL & 2) != 0) {
          asm volatile("" ::"v"(o.x), "v"(o.y));
        } else if (emit1) {
          *reinterpret_cast<double2 *>(dst + xo) = o;
        } else if (emit0) {
          dst[xo] = o.x;
        }
      }
      if ((i & (B - 1)) == B - 1) {
        // row i+B (issued in iteration i-D) landed; after it: D*G DMAs and
        // the stores of iterations i-D .. i (stores from iteration 4E+2B on)
        if (i - D >= 4 * E + 2 * B)
          wait_vmcnt<D * G + D + 1>();
        else
          wait_vmcnt<D * G>();
        row_barrier();
      }
    }
    wait_vmcnt<0>();
  }
}

template <int E, int ABL, int D = kPairD, bool SPLIT = false, int B = kPairSplitB>
int launch_pair_abl(const RectList &rl, const StepConst &c, hipStream_t st) {
  if constexpr (SPLIT)
    hipLaunchKernelGGL((k_pair_split<E, D, ABL, B>), dim3(rl.nwork), dim3(128), 0, st, rl, c);
  else
    hipLaunchKernelGGL((k_pair<E, D, ABL>), dim3(rl.nwork), dim3(64), 0, st, rl, c);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace nlh
