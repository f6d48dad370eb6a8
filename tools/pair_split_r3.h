// pair_split_r3.h -- frozen round-3 k_pair_split (one row per scatter), kept for
// the tools/pair_bench.hip comparison with the row-pair kernel of nlh_pair.h.
#pragma once
#include "nlh_pair.h"
namespace nlh {
// Nested windows of the lane's two columns scattered into the accumulators
// of the 2E+1 output rows this input row touches (slot of output row
// input+d = (QA + d) mod P; QA = the input row's own slot), plus the folded
// centre term.
template <int E, int QA>
__device__ __forceinline__ void pair_scatter_r3(const double (&w)[2 * E + 2], double (&acc)[2][2 * E + 1],
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
template <int E, int D, int ABL = 0, int B = kPairSplitB, bool TEST = false>
__global__ __launch_bounds__(128, 2) void k_pair_split_r3(RectList L, StepConst C) {
  constexpr int R = 2;
  constexpr int P = 2 * E + 1;
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

  // barriers: one prologue barrier, then one after every iteration i with
  // i % B == B-1, for i = 0 .. i_last (wave 0 stops computing at n_in - 1)
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
        constexpr int so = (q + E + 1) % P;
        const int i = b + q;
        if constexpr ((ABL & 32) == 0)
          if (i >= n_in) return;
        double w[NW];
        window(ring + ((bs + q) & (K - 1)) * RW + R * lane, w);
        pair_scatter_r3<E, q>(w, acc, kc);
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
    int row = 0;  // next u^t row to fetch (clamped at the last one)
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
      if constexpr ((ABL & 32) != 0)
        gnext += stride;
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
    for (int b = P; b <= i_last; b += P) {
      auto body = [&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int q2 = ((q + 1 - B) % P + P) % P;  // slot of row m2 = i - 2E - B
        constexpr int so = (q2 + E + 1) % P;
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
        pair_scatter_r3<E, q2>(w2, acc, kc);
        if constexpr (TEST) {  // (dt/alpha) b(t+1) at the centre row of the output
          const double *qr = qbuf + (m2 & (U1R - 1)) * U1W + R * lane + E;
          acc[0][q2] += qr[0];
          acc[1][q2] += qr[1];
        }
        if ((ABL & 32) != 0 || m2 >= 2 * E) {
          const double o0 = alpha * acc[0][so];
          const double o1 = alpha * acc[1][so];
          double *dst = run + (int64_t)(yout0 + ydir * (m2 - 2 * E)) * pitch;
          if constexpr ((ABL & 2) != 0 || (ABL & 128) != 0) {
            asm volatile("" ::"v"(o0), "v"(o1));
          } else if constexpr ((ABL & 512) != 0) {  // ablation: non-temporal stores
            if (emit1) {
              __builtin_nontemporal_store(o0, dst + xo);
              __builtin_nontemporal_store(o1, dst + xo + 1);
            } else if (emit0) {
              __builtin_nontemporal_store(o0, dst + xo);
            }
          } else if (emit1) {
            *reinterpret_cast<double2 *>(dst + xo) = make_double2(o0, o1);
          } else if (emit0) {
            dst[xo] = o0;
          }
        }
        if constexpr ((ABL & 40) != 40) block_end(i);
      };
      static_for<P>(body);
      bs = (bs + P) & (K - 1);
    }
    wait_vmcnt<0>();  // drain the clamped tail DMAs and the stores
  }
}
}  // namespace nlh
