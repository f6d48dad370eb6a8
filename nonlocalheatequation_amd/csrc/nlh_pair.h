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
//            finished row is written to a one-row LDS buffer;
//   stage 2: the same sweep over that u^{t+1} row, emitting u^{t+2} for the
//            64R-2E columns x0 .. x0+64R-2E and rows Y0 .. Y1.
//
// u^{t+1} never touches HBM: per two steps the kernel reads u^t (with a 2E
// halo) and writes u^{t+2} once, about half the single-step traffic.
//
// Centre fold: u' = u + alpha*(S - N u) = alpha*(S + (1/alpha - N) u), so the
// centre value is added to its own accumulator (kc = 1/alpha - N) when its row
// arrives and no centre rows have to be kept.  The extra rounding is a few ulp
// of the field scale; alpha == 0 never reaches this kernel.
#pragma once

#include "nlh_device.h"
#include "nlh_kernel_common.h"

namespace nlh {

constexpr int kPairD = 6;  // u^t rows in flight per wave

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

// nested windows H_L (L = 0..E) of the lane's R columns, scattered into the
// accumulators of the 2E+1 output rows this input row touches; QA = the
// input row's own slot.  Plus the folded centre term.
template <int E, int R, int QA>
__device__ __forceinline__ void pair_scatter(const double (&w)[R + 2 * E], double (&acc)[R][2 * E + 1],
                                             double kc) {
  constexpr int P = 2 * E + 1;
#pragma unroll
  for (int c = 0; c < R; ++c) {
    double h = w[E + c];
#pragma unroll
    for (int Lv = 0; Lv <= E; ++Lv) {
      if (Lv > 0) h = h + (w[E + c - Lv] + w[E + c + Lv]);
#pragma unroll
      for (int d = -E; d <= E; ++d) {
        if (clen(E, d < 0 ? -d : d) == Lv) acc[c][(QA + d + P) % P] += h;
      }
    }
    acc[c][QA] = fma(kc, w[E + c], acc[c][QA]);
  }
}

// ABL (diagnostics only, NLH_PAIR_ABLATE): bit mask, 0 = production.
// 2 = no HBM traffic (no DMA, no stores), 16 = no u^t window LDS reads,
// 32 = no u^{t+1} LDS write/window reads
template <int E, int D, int ABL = 0>
__global__ __launch_bounds__(64) void k_pair(RectList L, StepConst C) {
  constexpr int R = 2;
  constexpr int P = 2 * E + 1;
  constexpr int W1 = 64 * R;          // u^{t+1} columns per strip
  constexpr int WO = W1 - 2 * E;      // output columns per strip
  constexpr int RW = W1 + 2 * E;      // staged u^t doubles per ring row
  constexpr int NCH = RW / 2;         // 16-byte chunks per row
  constexpr int K = pow2_ceil(D + 1); // ring slots
  constexpr int G = (NCH + 63) / 64;  // DMA instructions per row
  constexpr int U1W = W1 + 2 * E + 2; // u^{t+1} row + read-over pad (lanes >= WO/R)
  // stores count in vmcnt (see k_fast); lane 0 always owns an output column
  static_assert(D * G + D < 64, "vmcnt range");
  static_assert(WO >= 64, "strip too narrow for this eps");

  __shared__ __attribute__((aligned(16))) double ring[K * RW + U1W];
  double *const u1row = ring + K * RW;

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

  bool cin[R];  // this lane's u^{t+1} columns lie inside the lattice
#pragma unroll
  for (int c = 0; c < R; ++c) {
    const int gx = rgx0 + x0 - E + R * lane + c;
    cin[c] = gx >= 0 && gx < (int)C.nx;
  }
  const int xo = x0 + R * lane;  // first output column of this lane
  const bool emit0 = R * lane < WO && xo < rx1;
  const bool emit1 = R * lane < WO && xo + 1 < rx1;
  double *dst = run + (int64_t)(up ? Y1 - 1 : Y0) * pitch + xo;

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

  int bs = 0;  // b % K
  for (int b = 0; b < n_in; b += P) {
    // static unroll over the accumulator period: every slot index below is a
    // compile-time constant, so acc1/acc2 stay in registers
    auto body = [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const int i = b + q;
      if (i >= n_in) return;
      const int slot = (bs + q) & (K - 1);
      issue(i + D, (bs + q + D) & (K - 1));
      if (i >= 4 * E + D)
        wait_vmcnt<D * G + D>();
      else
        wait_vmcnt<D * G>();

      // stage 1: u^t row i into acc1
      double w[R + 2 * E];
      if constexpr ((ABL & 16) != 0) {
#pragma unroll
        for (int k = 0; k < R + 2 * E; ++k) w[k] = (double)(k + i);
      } else {
        pair_window<E, R>(ring + slot * RW + R * lane, w);
      }
      pair_scatter<E, R, q>(w, acc1, kc);
      constexpr int so1 = (q + E + 1) % P;  // u^{t+1} row of input row i-E done
      if (i >= 2 * E) {
        const int m = i - 2 * E;
        const int gy = gy1first + ydir * m;
        const bool rin = gy >= 0 && gy < gny;
        double v[R];
#pragma unroll
        for (int c = 0; c < R; ++c) v[c] = (rin && cin[c]) ? alpha * acc1[c][so1] : 0.0;
        // stage 2: u^{t+1} row m into acc2 (m = i - 2E, so m mod P = q + 1)
        constexpr int q2 = (q + 1) % P;
        constexpr int so2 = (q2 + E + 1) % P;
        double w2[R + 2 * E];
        if constexpr ((ABL & 32) != 0) {
#pragma unroll
          for (int k = 0; k < R + 2 * E; ++k) w2[k] = v[k & 1] + (double)k;
        } else {
          asm volatile("" ::: "memory");  // previous row's window reads stay before this write
          *reinterpret_cast<double2 *>(u1row + R * lane) = make_double2(v[0], v[1]);
          asm volatile("" ::: "memory");  // LDS is in order per wave: reads see every lane's write
          pair_window<E, R>(u1row + R * lane, w2);
        }
        pair_scatter<E, R, q2>(w2, acc2, kc);
        if (i >= 4 * E) {
          const double o0 = alpha * acc2[0][so2];
          const double o1 = alpha * acc2[1][so2];
          if constexpr ((ABL & 2) != 0) {
            asm volatile("" ::"v"(o0), "v"(o1));
          } else if (emit1) {
            *reinterpret_cast<double2 *>(dst) = make_double2(o0, o1);
          } else if (emit0) {
            dst[0] = o0;
          }
          dst += stride;
        }
#pragma unroll
        for (int c = 0; c < R; ++c) acc2[c][so2] = 0.0;
      }
#pragma unroll
      for (int c = 0; c < R; ++c) acc1[c][so1] = 0.0;
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

template <int E>
int launch_pair_e(const RectList &rl, const StepConst &c, hipStream_t st) {
  hipLaunchKernelGGL((k_pair<E, kPairD>), dim3(rl.nwork), dim3(64), 0, st, rl, c);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace nlh
