// nlh_prefix.hip -- instances and launcher of k_prefix_rt (nlh_prefix.h).
#include "nlh_prefix.h"

#include <cstdlib>

namespace nlh {

// 65 .. 224: one staged chunk (k_prefix_rt); past 224 the chunked k_prefix_rtc
// up to kPrefixMaxE (its LDS: 2 (64 x 8 x nchk + 2) doubles, nchk <= 19:
// <= 152 KB, one workgroup per CU at the largest horizons)
bool prefix_rt_supported(int E) { return E >= 65 && E <= kPrefixMaxE; }

// chunks of 64 x 8 columns k_prefix_rtc / k_prefix_rtw stage (64 W + 2E
// rounded up to even)
static int prefix_rtc_chunks(int E, int W = 1) { return (64 * W + 2 * E + (E & 1) * 2 + 511) / 512; }

int prefix_rt_window(int E, int W) { return E <= 224 && W == 1 ? 512 : 512 * prefix_rtc_chunks(E, W); }

bool prefix_rt_waves_ok(int E, int W) {
  if (W == 1) return true;
  return (W == 2 || W == 4 || W == 8 || W == 16) && prefix_rtc_chunks(E, W) <= kPrefixMaxChunks;
}

// W and R by E (round 6; tools/gpu/r6_prefix_{rows,waves,grid}.sh,
// profiles/r06/prefix_rows/, G node-updates/s on one box):
// * k_prefix_rt (W = 1, R = 32, partial-horizon rows peeled) up to eps 160:
//   eps 65 / 96 / 130 34.2 / 23.6 / 17.5 against 25.4 / 18.6 / 12.5 for the
//   best shared-row form -- its pair loop dominates its one-chunk scan;
// * W = 16, R = 32 from 161 to 1800 (eps 200 8.49 against 6.89; 300 5.07
//   against 2.39 for round 5's k_prefix_rtc; 600 2.34; 1500 0.709);
// * W = 8, R = 32 past 1800 while its window fits the LDS (eps 2000 / 3000 /
//   4000: 0.245 / 0.126 / 0.077 against 0.229 / 0.115 / 0.072 at W = 16);
// * then W = 4, 2 (R = 64), and W = 1 (R = 128: one workgroup per CU by LDS,
//   accumulators partly in AGPRs) up to 4832.
// Fewer rows per work item pay as W grows: the scan is shared by the waves,
// and R = 32 keeps ~100 VGPRs (four waves per SIMD)
int prefix_rt_waves(int E) {
  if (const char *v = std::getenv("NLH_PREFIX_WAVES"))
    if (*v && std::atoi(v) != 0) return std::atoi(v);
  if (E <= 160) return 1;
  for (int W : {E <= 1800 ? 16 : 8, 4, 2})
    if (prefix_rtc_chunks(E, W) <= kPrefixMaxChunks) return W;
  return 1;
}

int prefix_rt_rows(int E, int W) {
  if (const char *v = std::getenv("NLH_PREFIX_ROWS"))
    if (*v && std::atoi(v) != 0) return std::atoi(v);
  if (W >= 8 || E <= 224) return kPrefixRows;
  if (W > 1) return 64;
  return prefix_rtc_chunks(E) >= 10 ? 128 : 96;
}

int prefix_rt_table_size(int E, int R) { return 2 * (E + R) + 1; }


// columns per lane of the launched instances (launch_prefix_rt)
static int prefix_rt_cpl(int) { return 1; }
int prefix_rt_strip_width(int E, int W) { return 64 * prefix_rt_cpl(E) * W; }

void prefix_rt_table(int E, int R, const int32_t *lens, int32_t *out) {
  for (int i = 0; i < prefix_rt_table_size(E, R); ++i) {
    const int d = i - E - R;
    const int ad = d < 0 ? -d : d;
    out[2 * i] = ad <= E ? lens[ad] : 0;
    out[2 * i + 1] = ad <= E ? -lens[ad] - 1 : 0;
  }
}

template <int NV, bool TEST, int R>
static int launch_nv_r(const RectList &rl, const StepConst &c, const void *table, hipStream_t st) {
  hipLaunchKernelGGL((k_prefix_rt<NV, R, TEST, false, false, 1, true>), dim3(rl.nwork), dim3(64), 0, st, rl,
                     c, (const int2 *)table);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// R from the rect list (every rect of a prefix list has seg_rows == R)
template <int NV, bool TEST>
static int launch_nv(const RectList &rl, const StepConst &c, const void *table, hipStream_t st) {
  return rl.r[0].seg_rows == 64 ? launch_nv_r<NV, TEST, 64>(rl, c, table, st)
                                : launch_nv_r<NV, TEST, kPrefixRows>(rl, c, table, st);
}

template <int R>
static int launch_rtc(const RectList &rl, const StepConst &c, const void *table, bool test, int nchk, size_t lds,
                      hipStream_t st) {
  if (test)
    hipLaunchKernelGGL((k_prefix_rtc<8, R, true>), dim3(rl.nwork), dim3(64), lds, st, rl, c, (const int2 *)table, nchk);
  else
    hipLaunchKernelGGL((k_prefix_rtc<8, R, false>), dim3(rl.nwork), dim3(64), lds, st, rl, c, (const int2 *)table, nchk);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

bool prefix_rt_rows_ok(int E, int R) {
  return R == 32 || R == 64 || (E > 224 && (R == 96 || R == 128));
}

template <int R, int W>
static int launch_rtw(const RectList &rl, const StepConst &c, const void *table, bool test, int nchk, size_t lds,
                      hipStream_t st) {
  if (test)
    hipLaunchKernelGGL((k_prefix_rtw<8, R, true, W>), dim3(rl.nwork), dim3(64 * W), lds, st, rl, c,
                       (const int2 *)table, nchk);
  else
    hipLaunchKernelGGL((k_prefix_rtw<8, R, false, W>), dim3(rl.nwork), dim3(64 * W), lds, st, rl, c,
                       (const int2 *)table, nchk);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

template <int W>
static int launch_rtw_r(const RectList &rl, const StepConst &c, const void *table, bool test, int nchk,
                        hipStream_t st) {
  const size_t lds = (2 * (size_t)(512 * nchk + 2) + 2 * (size_t)nchk) * sizeof(double);
  switch (rl.r[0].seg_rows) {
    case 32: return launch_rtw<32, W>(rl, c, table, test, nchk, lds, st);
    case 64: return launch_rtw<64, W>(rl, c, table, test, nchk, lds, st);
    case 96: return launch_rtw<96, W>(rl, c, table, test, nchk, lds, st);
    case 128: return launch_rtw<128, W>(rl, c, table, test, nchk, lds, st);
  }
  return -1;
}

int launch_prefix_rt(const RectList &rl, const StepConst &c, const void *table, bool test, int waves, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (rl.nwork <= 0) return 0;
  if (c.E > kPrefixMaxE) return -1;
  if (waves > 1) {
    const int nw = prefix_rtc_chunks(c.E, waves);
    if (nw > kPrefixMaxChunks) return -1;
    switch (waves) {
      case 2: return launch_rtw_r<2>(rl, c, table, test, nw, st);
      case 4: return launch_rtw_r<4>(rl, c, table, test, nw, st);
      case 8: return launch_rtw_r<8>(rl, c, table, test, nw, st);
      case 16: return launch_rtw_r<16>(rl, c, table, test, nw, st);
    }
    return -1;
  }
  // the staged window 64 + 2E (rounded up to even) <= 64 NV columns; the
  // narrowest NV that holds it (every staged value is loaded, scanned and
  // written to LDS: eps 97 ran at 12.8 G node/s with NV = 8 against 23.4 G
  // at eps 96 with NV = 4, profiles/r04/first/)
  if (c.E <= 96) return test ? launch_nv<4, true>(rl, c, table, st) : launch_nv<4, false>(rl, c, table, st);
  if (c.E <= 160) return test ? launch_nv<6, true>(rl, c, table, st) : launch_nv<6, false>(rl, c, table, st);
  if (c.E <= 224) return test ? launch_nv<8, true>(rl, c, table, st) : launch_nv<8, false>(rl, c, table, st);
  const int nchk = prefix_rtc_chunks(c.E);
  if (nchk > kPrefixMaxChunks) return -1;
  const size_t lds = 2 * (size_t)(512 * nchk + 2) * sizeof(double);
  switch (rl.r[0].seg_rows) {
    case 32: return launch_rtc<32>(rl, c, table, test, nchk, lds, st);
    case 64: return launch_rtc<64>(rl, c, table, test, nchk, lds, st);
    case 96: return launch_rtc<96>(rl, c, table, test, nchk, lds, st);
    case 128: return launch_rtc<128>(rl, c, table, test, nchk, lds, st);
  }
  return -1;
}

}  // namespace nlh
