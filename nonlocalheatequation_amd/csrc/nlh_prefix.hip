// nlh_prefix.hip -- instances and launcher of k_prefix_rt (nlh_prefix.h).
#include "nlh_prefix.h"

#include <cstdlib>

namespace nlh {

// 65 .. 224: one staged chunk (k_prefix_rt); past 224 the chunked k_prefix_rtc
// up to kPrefixMaxE (its LDS: 2 (64 x 8 x nchk + 2) doubles, nchk <= 19:
// <= 152 KB, one workgroup per CU at the largest horizons)
bool prefix_rt_supported(int E) { return E >= 65 && E <= kPrefixMaxE; }

// chunks of 64 x 8 columns k_prefix_rtc stages (64 + 2E rounded up to even)
static int prefix_rtc_chunks(int E) { return (64 + 2 * E + (E & 1) * 2 + 511) / 512; }

int prefix_rt_window(int E) { return E <= 224 ? 512 : 512 * prefix_rtc_chunks(E); }

int prefix_rt_table_size(int E, int R) { return 2 * (E + R) + 1; }

// by E (round 6, tools/gpu/r6_prefix_rows.sh, profiles/r06/prefix_rows/): at
// eps 96 R = 64 ran as R = 32 and at 160 8% slower (k_prefix_rt's pair loop
// dominates its short scan); the chunked kernel's scan of the 64 + 2E-column
// window is shared by R output rows: R = 96 (242 VGPRs, two waves per SIMD)
// beat 64 by 11-26% at eps 300-1500, R = 128 (accumulators partly in AGPRs,
// one wave per SIMD) lost there but won by 21% at eps 4832, where the LDS
// already holds one workgroup per CU -- so 128 from 10 chunks (>= 80 KB of LDS)
int prefix_rt_rows(int E) {
  if (const char *v = std::getenv("NLH_PREFIX_ROWS"))
    if (*v && std::atoi(v) != 0) return std::atoi(v);
  if (E <= 224) return kPrefixRows;
  return prefix_rtc_chunks(E) >= 10 ? 128 : 96;
}

// columns per lane of the launched instances (launch_prefix_rt)
static int prefix_rt_cpl(int) { return 1; }
int prefix_rt_strip_width(int E) { return 64 * prefix_rt_cpl(E); }

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

int launch_prefix_rt(const RectList &rl, const StepConst &c, const void *table, bool test, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (rl.nwork <= 0) return 0;
  // the staged window 64 + 2E (rounded up to even) <= 64 NV columns; the
  // narrowest NV that holds it (every staged value is loaded, scanned and
  // written to LDS: eps 97 ran at 12.8 G node/s with NV = 8 against 23.4 G
  // at eps 96 with NV = 4, profiles/r04/first/)
  if (c.E <= 96) return test ? launch_nv<4, true>(rl, c, table, st) : launch_nv<4, false>(rl, c, table, st);
  if (c.E <= 160) return test ? launch_nv<6, true>(rl, c, table, st) : launch_nv<6, false>(rl, c, table, st);
  if (c.E <= 224) return test ? launch_nv<8, true>(rl, c, table, st) : launch_nv<8, false>(rl, c, table, st);
  if (c.E > kPrefixMaxE) return -1;
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
