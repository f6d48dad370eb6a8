// nlh_wide_rt.h -- large-horizon single step with a RUN-TIME horizon,
// k_wide_rt (J = 1, eps 49 .. 64): the reference's sum_local
// (src/2d_nonlocal_serial.cpp:256-270; update :279-284) past the compile-time
// k_wide instances (nlh_wide.h, eps <= 48), O(eps) work per node instead of
// the direct O(eps^2) disk sum of k_exact.
//
// Layout as k_wide with prefix-sum rows built PA rows ahead (nlh_wide.h PS /
// PA / PSPLIT): one 64-column strip per wave, input rows LDS-DMA'd D rows
// ahead, each staged row turned into its prefix row P by a DPP wave scan; the
// row window of half-width L at column c is P(c+L) - P(c-L-1).  With E known
// only at run time, the disk level of each row offset d, len(d), is a run-time
// value: every d takes its own window (two ds_read_b64 at run-time offsets,
// one subtraction; len(d) broadcast from a small LDS table), and offsets past
// the horizon are masked to zero.
//
// The 2E+1 row offsets are split over TWO passes (two launches per step) so
// that each keeps only EMAX + CH accumulators live (two waves per SIMD, no
// AGPRs -- one pass with all 2*EMAX + CH spilled):
//   pass 0: dy in [-E, 0] -- slot a = c + d (d = -dy); the centre fold
//           (1/alpha - N) u and the test-mode source (dt/alpha) b; the partial
//           sum S0(k) is stored into the next-field buffer;
//   pass 1: dy in [1, E] -- slot a = c + EMAX - dy; u'(k) = alpha (S1(k) +
//           S0(k)), S0 read back from the next-field buffer (same lane, same
//           element) and overwritten.
// In chunk j (inputs i = CH*j + c, input i = block row Y0 - E + i) slots 0 ..
// CH-1 are complete after the chunk: output k = CH*j + a - E (pass 0) or
// CH*j + a - E - EMAX (pass 1); the block is then renamed a -> a - CH and its
// new slots zeroed.
#pragma once

#include "nlh_device.h"
#include "nlh_kernel_common.h"
#include "nlh_wide.h"

namespace nlh {

constexpr int kWideRtMax = 64;  // largest run-time horizon
constexpr int kWideRtMin = 49;  // smaller: the compile-time k_wide instances

template <int EMAX, int CH, bool TEST, int D, int PA, int PASS>
__global__ __launch_bounds__(64, 2) void k_wide_rt(RectList L, StepConst C) {
  constexpr int W = 64;                 // output columns per strip
  constexpr int EPM = (EMAX + 1) & ~1;  // staged halo columns per side, at most
  constexpr int RWM = W + 2 * EPM;      // staged doubles per ring row, at most
  constexpr int K = pow2_ceil(D + 1);   // ring slots
  // a u row is 64 + (NCH - 64) 16-byte chunks with NCH = 32 + EP in (64, 96]
  // for 33 <= E <= 64: two DMA instructions, the second on NCH - 64 lanes
  constexpr int GU = 2;
  constexpr bool SRC = TEST && PASS == 0;  // the manufactured source rides pass 0
  constexpr int GL = SRC ? (W / 2 + 63) / 64 : 0;
  constexpr int GS = SRC ? 1 : 0;
  constexpr int G = GU + GL + GS;
  constexpr int NA = EMAX + CH;  // live accumulators
  constexpr int PK = pow2_ceil(PA + 1);
  constexpr int NPR = RWM + 2;   // doubles per prefix slot: [1] = P(-1) = 0, [2 + k] = P(k)
  constexpr int GD = 4;          // row offsets per LDS read group (one 16-byte len(d) read)
  constexpr int D0 = PASS == 0 ? 0 : 1;                 // first row offset of this pass
  constexpr int NGD = (EMAX + 1 - D0 + GD - 1) / GD;   // groups
  static_assert(EMAX <= 64 && RWM <= 192, "two 16-byte chunks per lane cover a staged row");
  static_assert(D * G + CH < 64, "vmcnt range");
  static_assert(PA >= 1 && PA < D, "prefix rows ahead of the window reads, behind the DMA");

  __shared__ __attribute__((aligned(16))) double ring[K * RWM + (SRC ? K * W + 2 * K : 0) + PK * NPR];
  __shared__ __attribute__((aligned(16))) int lvt[NGD * GD];  // len(d0 + n), 0 past the horizon
  double *lwr = ring + K * RWM;  // L_h[W0] rows (test mode), same slots as the u rows
  double *syr = lwr + K * W;     // sin(2 pi y dh) pairs (test mode)
  double *pfx = ring + K * RWM + (SRC ? K * W + 2 * K : 0);

  const int lane = (int)threadIdx.x;
  const int E = C.E;  // host: kWideRtMin <= E <= EMAX
  const int EP = (E + 1) & ~1;
  const int NCH = 32 + EP;
  if (lane < PK) pfx[lane * NPR + 1] = 0.0;
  for (int n = lane; n < NGD * GD; n += 64) lvt[n] = D0 + n <= E ? C.lens[D0 + n] : 0;
  asm volatile("" ::: "memory");  // one wave: its LDS accesses are in order

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

  const int xl = x0 + lane;
  const bool emit = xl < rx1;
  double sxv = 0.0;
  if constexpr (SRC) sxv = C.sxt[rgx0 + min(xl, rx1 - 1) + E];

  const uint32_t lring = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  const uint32_t llw = __builtin_amdgcn_readfirstlane(lds_addr(lwr));
  const uint32_t lsy = __builtin_amdgcn_readfirstlane(lds_addr(syr));
  auto sy_index = [&](int i) {
    const int k = min(max(i - E, 0), nout - 1);
    return rgy0 + (up ? Y1 - 1 - k : Y0 + k) + E;
  };
  const double *gnext = ru + (int64_t)yfirst * pitch + (x0 - EP);
  const double *l0 = SRC ? Rc.lw + (int64_t)(up ? Y1 - 1 : Y0) * pitch + x0 : nullptr;
  int fetched = 0;
  auto issue = [&]() __attribute__((always_inline)) {
    const int slot = fetched & (K - 1);
    if constexpr (SRC) {
      const int k = min(fetched, n_in - 1) - E;
      dma_chunks<W / 2>(l0 + (int64_t)k * stride, llw + slot * W * 8, lane);
      dma_chunks<1>(C.syt + (sy_index(fetched) & ~1), lsy + slot * 16, lane);
    }
    const uint32_t dst = lring + slot * RWM * 8;
    dma16(gnext + 2 * lane, dst);
    if (lane < NCH - 64) dma16(gnext + 2 * (64 + lane), dst + 1024);
    ++fetched;
    if (fetched < n_in) gnext += stride;
  };
#pragma unroll
  for (int s = 0; s < D; ++s) issue();

  // prefix row of staged row r into prefix slot r mod PK
  auto scan_row = [&](int r) __attribute__((always_inline)) {
    const double *srow = ring + (r & (K - 1)) * RWM;
    double *dst = pfx + (r & (PK - 1)) * NPR + 2;
    const double2 ab = *reinterpret_cast<const double2 *>(srow + 2 * lane);
    double2 cd = make_double2(0.0, 0.0);
    if (lane < NCH - 64) cd = *reinterpret_cast<const double2 *>(srow + 2 * (lane + 64));
    const double sv = wave_prefix_sum(ab.x + ab.y);
    const double tot = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(sv), 63),
                                        __builtin_amdgcn_readlane(__double2loint(sv), 63));
    const double sw = wave_prefix_sum(cd.x + cd.y) + tot;
    asm volatile("" ::: "memory");
    *reinterpret_cast<double2 *>(dst + 2 * lane) = make_double2(sv - ab.y, sv);
    if (lane < NCH - 64) *reinterpret_cast<double2 *>(dst + 2 * (lane + 64)) = make_double2(sw - cd.y, sw);
    asm volatile("" ::: "memory");  // in order per wave: later reads see every lane's write
  };
  static_for<PA>([&](auto rc) __attribute__((always_inline)) {
    constexpr int r = decltype(rc)::value;
    wait_vmcnt<(D - 1 - r) * G>();
    scan_row(r);
  });

  double acc[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) acc[a] = 0.0;

  const double qs = SRC ? C.dt / alpha : 0.0;
  // outputs k = CH*j + a - KOFF; the last one, nout - 1, leaves slot range [0, CH) in chunk nchunk-1
  const int KOFF = PASS == 0 ? E : E + EMAX;
  const int nchunk = (nout - 1 + KOFF) / CH + 1;
  bool full = false;  // the previous chunk stored CH output rows
  for (int j = 0; j < nchunk; ++j) {
    const int ibase = j * CH;
    auto row = [&](auto cc) __attribute__((always_inline)) {
      constexpr int c = decltype(cc)::value;
      const int i = ibase + c;
      issue();  // input row i + D
      // row i + PA landed (issued after it: the DMAs of rows i+PA+1 .. i+D and,
      // for c + PA < D, the previous chunk's CH stores; pass 1's loads of S0 were waited for)
      if constexpr (c + PA < D) {
        if (full)
          wait_vmcnt<(D - PA) * G + CH>();
        else
          wait_vmcnt<(D - PA) * G>();
      } else {
        wait_vmcnt<(D - PA) * G>();
      }
      const double *pl = pfx + (i & (PK - 1)) * NPR + 2 + EP + lane;  // P(centre + k) at pl[k]
      double hp[2][GD], hm[2][GD];
      auto load = [&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value;
        const int4 la = *reinterpret_cast<const int4 *>(lvt + g * GD);
        const int lv[GD] = {la.x, la.y, la.z, la.w};
        static_for<GD>([&](auto tc) __attribute__((always_inline)) {
          constexpr int t = decltype(tc)::value;
          if constexpr (D0 + g * GD + t <= EMAX) {
            hp[g & 1][t] = pl[lv[t]];
            asm volatile("" ::: "memory");  // two ds_read_b64, not one 8-cycle ds_read2_b64
            hm[g & 1][t] = pl[-lv[t] - 1];
            asm volatile("" ::: "memory");
          }
        });
      };
      auto consume = [&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value;
        static_for<GD>([&](auto tc) __attribute__((always_inline)) {
          constexpr int t = decltype(tc)::value;
          constexpr int d = D0 + g * GD + t;
          if constexpr (d <= EMAX) {
            double h = hp[g & 1][t] - hm[g & 1][t];
            if constexpr (d >= kWideRtMin) h = d <= E ? h : 0.0;  // past the horizon
            // pinned where it is added: left free, the compiler sinks the adds
            // below every window read of the row and keeps all 2 (E+1) values
            // live (spills)
            constexpr int s = PASS == 0 ? c + d : c + EMAX - d;  // dy = -d / +d
            acc[s] += h;
            asm volatile("" : "+v"(acc[s]));
          }
        });
      };
      load(std::integral_constant<int, 0>{});
      scan_row(i + PA);  // independent of this row's windows: overlaps their reads
      static_for<NGD>([&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value;
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (g + 1 < NGD) load(std::integral_constant<int, g + 1>{});
        consume(gc);
      });
      if constexpr (PASS == 0) {
        const double wc = ring[(i & (K - 1)) * RWM + EP + lane];
        acc[c] = fma(kc, wc, acc[c]);  // centre fold: output k = i - E sits in slot c
        if constexpr (SRC) {
          const double syv = syr[2 * (i & (K - 1)) + (sy_index(i) & 1)];
          const double b = -(C.st2pi * (sxv * syv)) - C.ct * lwr[(i & (K - 1)) * W + lane];
          acc[c] = fma(qs, b, acc[c]);
        }
      }
    };
    static_for<CH>(row);
    // slots 0 .. CH-1 complete: output k = ibase + a - KOFF
    const int k0 = ibase - KOFF;
    full = k0 >= 0 && k0 + CH <= nout;
    static_for<CH>([&](auto ac) __attribute__((always_inline)) {
      constexpr int a = decltype(ac)::value;
      const int k = k0 + a;
      if (k >= 0 && k < nout && emit) {
        double *dst = run + (int64_t)(up ? Y1 - 1 - k : Y0 + k) * pitch + xl;
        if constexpr (PASS == 0)
          *dst = acc[a];                   // S0(k)
        else
          *dst = alpha * (acc[a] + *dst);  // alpha (S1 + S0)
      }
    });
    // rename: a -> a - CH; the block's new slots start at zero
#pragma unroll
    for (int a = 0; a < EMAX; ++a) acc[a] = acc[a + CH];
#pragma unroll
    for (int a = EMAX; a < NA; ++a) acc[a] = 0.0;
  }
  wait_vmcnt<0>();
}

// 8-row chunks; 4 in test mode's pass 0, whose source terms would otherwise
// push it past the 256 VGPRs of two waves per SIMD
constexpr int kWideRtD = 6;
constexpr int kWideRtPA = 2;
template <bool TEST, int PASS>
constexpr int wide_rt_chunk() { return TEST && PASS == 0 ? 4 : 8; }

template <bool TEST, int PASS>
int launch_wide_rt_p(const RectList &rl, const StepConst &c, hipStream_t st) {
  hipLaunchKernelGGL((k_wide_rt<kWideRtMax, wide_rt_chunk<TEST, PASS>(), TEST, kWideRtD, kWideRtPA, PASS>),
                     dim3(rl.nwork), dim3(64), 0, st, rl, c);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// both passes, in order on one stream: pass 1 reads what pass 0 stored
template <bool TEST>
int launch_wide_rt_t(const RectList &rl, const StepConst &c, hipStream_t st) {
  const int r = launch_wide_rt_p<TEST, 0>(rl, c, st);
  return r ? r : launch_wide_rt_p<TEST, 1>(rl, c, st);
}

// resident workgroups per CU of the heavier pass, for the host's segment height
template <bool TEST>
int wide_rt_blocks_per_cu_t() {
  int n = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &n, k_wide_rt<kWideRtMax, wide_rt_chunk<TEST, 0>(), TEST, kWideRtD, kWideRtPA, 0>, 64, 0);
  return e == hipSuccess ? n : 0;
}

}  // namespace nlh
