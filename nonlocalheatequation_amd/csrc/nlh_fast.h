// nlh_fast.h -- the production stencil kernel k_fast (see nlh_kernels.hip for
// the algorithm summary) and its launcher template.  Instantiated per horizon
// range in nlh_fast_e*.hip so the unrolled kernels build in parallel.
#pragma once
#include "nlh_kernel_common.h"

namespace nlh {

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
constexpr int kFastD = 6;  // rows in flight per wave

// ABL: timing-decomposition masks for the tools/ harness (tools/wide_bench.hip);
// libnlh instantiates ABL = 0 only (results are meaningless otherwise).  1 = no
// arithmetic (loads/stores kept, window values kept alive), 2 = no HBM traffic
// (no DMA, no stores), 4 = no XCD remap, 8 = no alternating sweep, 16 = no
// window LDS reads, 32 = plain (temporal) tail-chunk loads, 64 = plain loads
// everywhere, 128 = non-temporal stores
template <int E, int R, int D, bool TEST, int ABL = 0>
__global__ __launch_bounds__(64) void k_fast(RectList L, StepConst C) {
  constexpr int P = 2 * E + 1;          // accumulator period (static unroll)
  constexpr int W = 64 * R;             // strip width (outputs)
  constexpr int EP = (E + 1) & ~1;      // halo columns staged per side
  constexpr int RW = W + 2 * EP;        // doubles per ring row
  constexpr int NCH = RW / 2;           // 16-byte chunks per row
  // E > 12: the row ring no longer retains rows for the centre value; a compact
  // ring of E+1 centre rows (W doubles each) keeps LDS per wave small
  constexpr bool CR = (E > 12);
  constexpr int K = CR ? pow2_ceil(D + 1) : pow2_ceil(E + D + 1);  // ring slots (pow2)
  constexpr int KC = E + 1;             // centre-ring slots (CR)
  constexpr int GU = (NCH + 63) / 64;   // DMA instructions per u row
  constexpr int GL = TEST ? (W / 2 + 63) / 64 : 0;  // per L_h[W0] row
  // TEST: the sin(2 pi y dh) table entry of the row too, one 16-byte DMA: a
  // scalar load per row stalls the lone wave of a SIMD on every row (the
  // lgkmcnt wait for the LDS window also waits for it), 64% wait cycles
  constexpr int GS = TEST ? 1 : 0;
  constexpr int G = GU + GL + GS;
  constexpr int OFF = EP - E;           // window start inside a staged row
  static_assert(D >= 1, "prefetch distance");
  // gfx950 counts global stores in vmcnt too: once every one of the last D
  // iterations has emitted its output row (at least one store instruction each:
  // lane 0 always owns a column) the wait for row i admits D more ops
  static_assert(D * G + D < 64, "vmcnt range");

  __shared__ __attribute__((aligned(16))) double ring[K * RW + (TEST ? K * W + 2 * K : 0) + (CR ? KC * W : 0)];
  double *lwr = ring + K * RW;                          // L_h[W0] ring (TEST)
  double *syr = lwr + K * W;                            // sin(2 pi y dh) pairs (TEST)
  double *cring = ring + K * RW + (TEST ? K * W + 2 * K : 0);   // centre ring (CR)

  const int lane = (int)threadIdx.x;
  const int work = (ABL & 4) ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int ri = find_rect(L, work);
  // Rect / StepConst fields in locals (SGPRs): read through the kernarg
  // reference inside the loop they were re-loaded every row
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
  const int n_in = (Y1 - Y0) + 2 * E;   // input rows Y0-E .. Y1+E-1
  const bool up = !(ABL & 8) && (seg & 1) != 0;  // sweep direction
  const int64_t pitch = Rc.pitch;
  const int64_t stride = up ? -pitch : pitch;
  const int yfirst = up ? (Y1 + E - 1) : (Y0 - E);  // block-local row of input 0
  const double nf = C.nf, alpha = C.alpha;
  const bool wave_full = x0 + W <= rx1;  // every lane stores R columns

  const double *g0 = ru + (int64_t)yfirst * pitch + (x0 - EP);
  // L_h[W0] row of the output emitted at iteration j (j >= 2E): Y0 + j - 2E
  // sweeping down, Y1 - 1 - (j - 2E) sweeping up
  const double *l0 = TEST ? Rc.lw + (int64_t)(up ? Y1 - 1 : Y0) * pitch + x0 : nullptr;
  const uint32_t lring = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  const uint32_t llw = __builtin_amdgcn_readfirstlane(lds_addr(lwr));
  const uint32_t lsy = __builtin_amdgcn_readfirstlane(lds_addr(syr));
  // table index of sin(2 pi y dh) for the output of iteration i
  auto sy_index = [&](int i) {
    const int lr = min(max(i - 2 * E, 0), n_in - 2 * E - 1);
    return rgy0 + (up ? Y1 - 1 - lr : Y0 + lr) + E;
  };

  const int xl = x0 + R * lane;  // first column of this lane
  double sxv[R];
  if (TEST) {
#pragma unroll
    for (int c = 0; c < R; ++c) {
      const int xc = min(xl + c, rx1 - 1);
      sxv[c] = C.sxt[rgx0 + xc + E];
      asm volatile("" ::"v"(sxv[c]));  // wait for it before the DMA stream
    }
  }

  // u rows stream through a running pointer clamped at the last input row;
  // the L_h row for the output of iteration i is fetched with row i + D
  const double *gnext = g0;
  auto issue = [&](int i, int slot) {
    if (!(ABL & 2)) dma_chunks<NCH, !(ABL & 64), !(ABL & 96)>(gnext, lring + slot * RW * 8, lane);
    if (i + 1 < n_in) gnext += stride;
    if (TEST) {
      const int lr = min(max(i - 2 * E, 0), n_in - 2 * E - 1);
      dma_chunks<W / 2>(l0 + (int64_t)lr * stride, llw + slot * W * 8, lane);
      dma_chunks<1>(C.syt + (sy_index(i) & ~1), lsy + slot * 16, lane);
    }
  };

#pragma unroll
  for (int s = 0; s < D; ++s) issue(s, s);

  double acc[R][P];
#pragma unroll
  for (int c = 0; c < R; ++c)
#pragma unroll
    for (int j = 0; j < P; ++j) acc[c][j] = 0.0;
  double *dst = run + (int64_t)(up ? Y1 - 1 : Y0) * pitch + xl;  // output row of iteration 2E
  int bs = 0;     // b % K
  int cslot = 0;  // i % KC (CR)
  for (int b = 0; b < n_in; b += P) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const int i = b + q;
      if (i < n_in) {
        const int slot = (bs + q) & (K - 1);
        issue(i + D, (bs + q + D) & (K - 1));
        if (i >= 2 * E + D)
          wait_vmcnt<D * G + D>();
        else
          wait_vmcnt<D * G>();

        // window of this lane: columns xl-E .. xl+R-1+E
        double w[R + 2 * E];
        const double *rowp = ring + slot * RW;
        if constexpr ((ABL & 16) != 0) {
#pragma unroll
          for (int k = 0; k < R + 2 * E; ++k) w[k] = (double)k;
        } else if constexpr (R % 2 == 0) {  // 16-B aligned: R*lane and the staged row start are even
          constexpr int NB = (OFF + 2 * E + R + 1) / 2;
          const double2 *rp = reinterpret_cast<const double2 *>(rowp + R * lane);
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
          for (int k = 0; k < R + 2 * E; ++k) w[k] = rowp[OFF + R * lane + k];
        }
        if constexpr (CR) {
#pragma unroll
          for (int c = 0; c < R; ++c) cring[cslot * W + R * lane + c] = w[E + c];
        }

        // nested windows + scatter into the accumulators of rows i-d
        if (ABL & 1) {
#pragma unroll
          for (int k = 0; k < R + 2 * E; ++k) asm volatile("" ::"v"(w[k]));
        }
#pragma unroll
        for (int c = 0; c < R && !(ABL & 1); ++c) {
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
          double out[R];
          const double *crow = CR ? cring + (cslot + 1 == KC ? 0 : cslot + 1) * W + R * lane
                                  : ring + ((bs + q - E) & (K - 1)) * RW + EP + R * lane;
#pragma unroll
          for (int c = 0; c < R; ++c) {
            const double uc = crow[c];
            const double diff = fma(-nf, uc, acc[c][so]);
            out[c] = fma(diff, alpha, uc);
          }
          if (TEST) {
            const double syv = syr[2 * slot + (sy_index(i) & 1)];
            const double *lrow = lwr + slot * W + R * lane;
#pragma unroll
            for (int c = 0; c < R; ++c) {
              const double w0 = sxv[c] * syv;
              const double bsrc = -(C.st2pi * w0) - C.ct * lrow[c];
              out[c] = fma(bsrc, C.dt, out[c]);
            }
          }
          if constexpr ((ABL & 2) != 0) {
#pragma unroll
            for (int c = 0; c < R; ++c) asm volatile("" ::"v"(out[c]));
          } else if constexpr ((ABL & 128) != 0 && R == 2) {
            if (wave_full) {
              __builtin_nontemporal_store(out[0], dst);
              __builtin_nontemporal_store(out[1], dst + 1);
            } else if (xl + 1 < rx1) {
              *reinterpret_cast<double2 *>(dst) = make_double2(out[0], out[1]);
            } else if (xl < rx1) {
              dst[0] = out[0];
            }
          } else if constexpr (R == 2) {
            if (wave_full) {
              *reinterpret_cast<double2 *>(dst) = make_double2(out[0], out[1]);
            } else if (xl + 1 < rx1) {
              *reinterpret_cast<double2 *>(dst) = make_double2(out[0], out[1]);
            } else if (xl < rx1) {
              dst[0] = out[0];
            }
          } else {
#pragma unroll
            for (int c = 0; c < R; ++c)
              if (wave_full || xl + c < rx1) dst[c] = out[c];
          }
          dst += stride;
        }
#pragma unroll
        for (int c = 0; c < R; ++c) acc[c][so] = 0.0;
        if constexpr (CR) cslot = (cslot + 1 == KC) ? 0 : cslot + 1;
      }
    }
    bs = (bs + P) & (K - 1);
  }
  wait_vmcnt<0>();  // drain the clamped tail DMAs before the wave retires
}

template <int E, int R, bool TEST>
int launch_fast_er(const RectList &rl, const StepConst &c, hipStream_t st) {
  hipLaunchKernelGGL((k_fast<E, R, kFastD, TEST>), dim3(rl.nwork), dim3(64), 0, st, rl, c);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace nlh
