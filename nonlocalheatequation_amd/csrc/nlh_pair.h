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

constexpr int kPairD = 7;  // u^t rows in flight per wave (ring of 8 slots)

// some row offset d of the disk has half-width len(d) == L
__host__ __device__ constexpr bool pair_level_used(int E, int L) {
  for (int d = 0; d <= E; ++d)
    if (clen(E, d) == L) return true;
  return false;
}

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
// centre term.
template <int E, int QA>
__device__ __forceinline__ void pair_scatter(const double (&w)[2 * E + 2], double (&acc)[2][2 * E + 1],
                                             double kc) {
  constexpr int P = 2 * E + 1;
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
      auto tap = [&](auto dc) {
        constexpr int d = decltype(dc)::value - E;
        if constexpr (clen(E, d < 0 ? -d : d) == Lv) {
          acc[0][(QA + d + P) % P] += ha;
          acc[1][(QA + d + P) % P] += hb;
        }
      };
      static_for<P>(tap);
    }
  };
  static_for<E>(level);
  acc[0][QA] = fma(kc, w[E], acc[0][QA]);
  acc[1][QA] = fma(kc, w[E + 1], acc[1][QA]);
}

// ABL (diagnostics only, NLH_PAIR_ABLATE): 0 = production, 2 = no HBM
// traffic (no DMA, no stores; same instruction stream otherwise)
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
  const int seg_h = C.seg_pair;
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
      pair_scatter<E, q>(w2, acc2, kc);
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
      pair_scatter<E, q>(w, acc1, kc);
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

template <int E, int ABL, int D = kPairD>
int launch_pair_abl(const RectList &rl, const StepConst &c, hipStream_t st) {
  hipLaunchKernelGGL((k_pair<E, D, ABL>), dim3(rl.nwork), dim3(64), 0, st, rl, c);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// resident k_pair workgroups per CU (register/LDS-limited), for the
// host's choice of segment height
template <int E>
int pair_blocks_per_cu_e() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_pair<E, kPairD>, 64, 0) != hipSuccess) return 0;
  return n;
}

template <int E>
int launch_pair_e(const RectList &rl, const StepConst &c, hipStream_t st) {
  hipLaunchKernelGGL((k_pair<E, kPairD>), dim3(rl.nwork), dim3(64), 0, st, rl, c);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace nlh
