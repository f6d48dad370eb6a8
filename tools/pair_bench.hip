// pair_bench.hip -- standalone timing harness for two-step pass variants
// (nlh_pair.h) on one C2-sized block, without rebuilding libnlh.  Each
// variant advances the same field; results are compared bitwise with the
// first (reference) variant after the same number of passes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Inonlocalheatequation_amd/csrc \
//     -mllvm -pragma-unroll-threshold=1000000 tools/pair_bench.hip -o build/pair_bench
//   build/pair_bench [n=4096] [passes=200] [seg_rows=0: auto list]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>
#include <utility>

#include "nlh_pair.h"

using namespace nlh;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef void (*KFn)(RectList, StepConst);

struct Variant {
  const char *name;
  KFn fn;
  int threads;
  int wg_per_cu;  // resident workgroups per CU the segment height is sized for
  int strip_out;  // output columns per strip
};

constexpr int E = 8;

static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 4096;
  const int passes = argc > 2 ? std::atoi(argv[2]) : 200;
  const int seg_force = argc > 3 ? std::atoi(argv[3]) : 0;
  const int H = 2 * E, XL = 16;
  const int64_t pitch = ((XL + std::max<int64_t>(ceil_div(n, 256) * 256 + XL, n + 128)) + 7) / 8 * 8;
  const int64_t rows = n + 2 * (H + kPairPadRows);  // the library's pair-solver block layout
  const size_t bytes = (size_t)(pitch * rows) * sizeof(double);
  double *buf[2];
  for (auto &b : buf) {
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(b, 0, bytes));
  }
  std::vector<double> h((size_t)n * n);
  const double dh = 1.0 / n;
  for (int y = 0; y < n; ++y)
    for (int x = 0; x < n; ++x) h[(size_t)y * n + x] = std::sin(2 * M_PI * (x * dh)) * std::sin(2 * M_PI * (y * dh)) +
                                                      0.25 * std::sin(2 * M_PI * (7 * x * dh + 3 * y * dh));
  auto origin = [&](double *b) { return b + (int64_t)(H + kPairPadRows) * pitch + XL; };
  int disk = 0;
  for (int d = -E; d <= E; ++d) disk += 2 * clen(E, d < 0 ? -d : d) + 1;
  StepConst C{};
  const double dt = std::pow((double)E, 4) * dh * dh / (8.0 * disk);
  C.c2d = 8.0 / std::pow(E * dh, 4);
  C.dh2 = dh * dh;
  C.dt = dt;
  C.alpha = C.c2d * C.dh2 * dt;
  C.nf = disk;
  C.kc = 1.0 / C.alpha - disk;
  C.nx = n;
  C.ny = n;
  C.E = E;

  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;

  // ablation masks of k_pair_split (nlh_pair.h): 4 no LDS window reads,
  // 8 no s_barrier, 16 no u^{t+1} LDS writes, 32 no checks, 64 no vmcnt
  // wait, 128 no store, 256 no DMA, 512 nt stores, 1024 nt DMA; 452 = VALU
  // only (no LDS reads, no vmcnt waits, no stores, no DMA)
  // OPT (nlh_pair.h): 1 incremental output row pointer, 2 unclamped row DMA,
  // 4 uniform single-column store, 8 wave 1 at wave priority 3
#if defined(PB_SET_TRACE)
  // -DPB_SET_TRACE: one launch of each variant with ABL 2048 (per-wave HW_ID,
  // XCC_ID and s_memrealtime entry / exit stamps); summary on stdout, raw
  // records to PB_TRACE_OUT (default pair_trace_<variant>.csv)
  std::vector<Variant> vs = {
      {"opt15", k_pair_split<E, 4, 2048, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt31", k_pair_split<E, 4, 2048, 2, false, 31>, 128, 4, 128 - 2 * E},
      {"opt7", k_pair_split<E, 4, 2048, 2, false, 7>, 128, 4, 128 - 2 * E},
      {"opt63", k_pair_split<E, 4, 2048, 2, false, 63>, 128, 4, 128 - 2 * E},
      {"opt223", k_pair_split<E, 4, 2048, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt223_D8", k_pair_split<E, 8, 2048, 2, false, 223>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_HEAD)
  // -DPB_SET_HEAD: OPT 15 (round-4 library) against 31 (head taps left out), interleaved
  std::vector<Variant> vs = {
      {"opt15", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt31", k_pair_split<E, 4, 0, 2, false, 31>, 128, 4, 128 - 2 * E},
      {"opt15_b", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt31_b", k_pair_split<E, 4, 0, 2, false, 31>, 128, 4, 128 - 2 * E},
      {"opt15_c", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt31_c", k_pair_split<E, 4, 0, 2, false, 31>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_PF)
  // -DPB_SET_PF: OPT 15 against 47 (within-block window prefetch), 63 (+ head skip)
  std::vector<Variant> vs = {
      {"opt15", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt47", k_pair_split<E, 4, 0, 2, false, 47>, 128, 4, 128 - 2 * E},
      {"opt63", k_pair_split<E, 4, 0, 2, false, 63>, 128, 4, 128 - 2 * E},
      {"opt15_b", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt47_b", k_pair_split<E, 4, 0, 2, false, 47>, 128, 4, 128 - 2 * E},
      {"opt63_b", k_pair_split<E, 4, 0, 2, false, 63>, 128, 4, 128 - 2 * E},
      {"opt39_b", k_pair_split<E, 4, 0, 2, false, 39>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_OCC)
  // -DPB_SET_OCC: workgroups per CU the segment height is sized for (1, 2: the
  // latency-bound rate of one / two waves per SIMD; 6, 8: three / four waves)
  std::vector<Variant> vs = {
      {"opt15_w4", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt15_w1", k_pair_split<E, 4, 0, 2, false, 15>, 128, 1, 128 - 2 * E},
      {"opt15_w2", k_pair_split<E, 4, 0, 2, false, 15>, 128, 2, 128 - 2 * E},
      {"opt15_w6", k_pair_split<E, 4, 0, 2, false, 15>, 128, 6, 128 - 2 * E},
      {"opt15_w8", k_pair_split<E, 4, 0, 2, false, 15>, 128, 8, 128 - 2 * E},
      {"opt7_w8", k_pair_split<E, 4, 0, 2, false, 7>, 128, 8, 128 - 2 * E},
      {"opt63_w6", k_pair_split<E, 4, 0, 2, false, 63>, 128, 6, 128 - 2 * E},
      {"opt63_w4", k_pair_split<E, 4, 0, 2, false, 63>, 128, 4, 128 - 2 * E},
      {"opt15_w4b", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_PI)
  // -DPB_SET_PI: OPT 15 / 63 against 79 / 95 (row pairs' levels interleaved)
  std::vector<Variant> vs = {
      {"opt15", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt63", k_pair_split<E, 4, 0, 2, false, 63>, 128, 4, 128 - 2 * E},
      {"opt79", k_pair_split<E, 4, 0, 2, false, 79>, 128, 4, 128 - 2 * E},
      {"opt95", k_pair_split<E, 4, 0, 2, false, 95>, 128, 4, 128 - 2 * E},
      {"opt15_b", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt63_b", k_pair_split<E, 4, 0, 2, false, 63>, 128, 4, 128 - 2 * E},
      {"opt79_b", k_pair_split<E, 4, 0, 2, false, 79>, 128, 4, 128 - 2 * E},
      {"opt95_b", k_pair_split<E, 4, 0, 2, false, 95>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_ABL)
  // -DPB_SET_ABL: ablations of OPT 15 (nlh_pair.h ABL bits; results not
  // meaningful): 4 no LDS window reads, 8 no s_barrier, 64 no vmcnt waits,
  // 72 neither, 2 no HBM traffic, 452 VALU only
  std::vector<Variant> vs = {
      {"abl0", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"abl4", k_pair_split<E, 4, 4, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"abl8", k_pair_split<E, 4, 8, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"abl64", k_pair_split<E, 4, 64, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"abl72", k_pair_split<E, 4, 72, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"abl2", k_pair_split<E, 4, 2, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"abl452", k_pair_split<E, 4, 452, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"abl460", k_pair_split<E, 4, 460, 2, false, 15>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_TAIL)
  // -DPB_SET_TAIL: OPT 15 (round 4), 31 (head), 95 (head + interleave), 223 (+ tail)
  std::vector<Variant> vs = {
      {"opt15", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt31", k_pair_split<E, 4, 0, 2, false, 31>, 128, 4, 128 - 2 * E},
      {"opt95", k_pair_split<E, 4, 0, 2, false, 95>, 128, 4, 128 - 2 * E},
      {"opt223", k_pair_split<E, 4, 0, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt159", k_pair_split<E, 4, 0, 2, false, 159>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_DEPTH)
  // -DPB_SET_DEPTH: DMA rows in flight (D) under OPT 223, barrier block 2
  std::vector<Variant> vs = {
      {"opt223_D4", k_pair_split<E, 4, 0, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt223_D6", k_pair_split<E, 6, 0, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt223_D8", k_pair_split<E, 8, 0, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt223_D12", k_pair_split<E, 12, 0, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt15_D4", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt15_D8", k_pair_split<E, 8, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_LEAN)
  // -DPB_SET_LEAN: OPT 15, 95, 223 against the lean periods 351 (95|256), 479 (223|256)
  std::vector<Variant> vs = {
      {"opt15", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt95", k_pair_split<E, 4, 0, 2, false, 95>, 128, 4, 128 - 2 * E},
      {"opt223", k_pair_split<E, 4, 0, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt351", k_pair_split<E, 4, 0, 2, false, 351>, 128, 4, 128 - 2 * E},
      {"opt479", k_pair_split<E, 4, 0, 2, false, 479>, 128, 4, 128 - 2 * E},
      {"opt415", k_pair_split<E, 4, 0, 2, false, 415>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_NOP)
  // -DPB_SET_NOP: OPT 223 with eight s_nop per row added on wave 0 (4096) or
  // wave 1 (8192): what non-VALU instructions on each role's path cost
  std::vector<Variant> vs = {
      {"opt223", k_pair_split<E, 4, 0, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt223_nop0", k_pair_split<E, 4, 4096, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt223_nop1", k_pair_split<E, 4, 8192, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt223_nop01", k_pair_split<E, 4, 12288, 2, false, 223>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_W0)
  // -DPB_SET_W0: wave 0 (stage 1) is the critical role under OPT 223
  // (profiles/r05/nop): its priority (8 off: 215; 512: wave 0 at priority 3
  // instead of wave 1: 735) and stage-1 lean periods (256: 479, 471, 991)
  std::vector<Variant> vs = {
      {"opt223", k_pair_split<E, 4, 0, 2, false, 223>, 128, 4, 128 - 2 * E},
      {"opt215", k_pair_split<E, 4, 0, 2, false, 215>, 128, 4, 128 - 2 * E},
      {"opt735", k_pair_split<E, 4, 0, 2, false, 735>, 128, 4, 128 - 2 * E},
      {"opt479", k_pair_split<E, 4, 0, 2, false, 479>, 128, 4, 128 - 2 * E},
      {"opt471", k_pair_split<E, 4, 0, 2, false, 471>, 128, 4, 128 - 2 * E},
      {"opt991", k_pair_split<E, 4, 0, 2, false, 991>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_RING)
  // -DPB_SET_RING: OPT 479 (round-5 library) against 2527 (+ period-aligned rings)
  std::vector<Variant> vs = {
      {"opt479", k_pair_split<E, 4, 0, 2, false, 479>, 128, 4, 128 - 2 * E},
      {"opt2527", k_pair_split<E, 4, 0, 2, false, 2527>, 128, 4, 128 - 2 * E},
      {"opt15", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt2063", k_pair_split<E, 4, 0, 2, false, 2063>, 128, 4, 128 - 2 * E},
      {"opt6623", k_pair_split<E, 4, 0, 2, false, 6623>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_ONE)
  // -DPB_SET_ONE: the production pass alone (compiler-option A/B: one binary per option)
  std::vector<Variant> vs = {
      {PB_NAME, k_pair_split<E, 4, 0, 2, false, 6623>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_TESTABL)
  // -DPB_SET_TESTABL: the test-mode pass with and without its L_h[W0] row DMA
  // (ablation 16384; results not meaningful), with the separable L_h[W0]
  // (OPT 32768: the library's E = 8 default from round 5), beside the
  // production pass
  std::vector<Variant> vs = {
      {"test", k_pair_split<E, 4, 0, 2, true, 6623>, 128, 4, 128 - 2 * E},
      {"test_nolw", k_pair_split<E, 4, 16384, 2, true, 6623>, 128, 4, 128 - 2 * E},
      {"test_sep", k_pair_split<E, 4, 0, 2, true, 6623 | 32768>, 128, 4, 128 - 2 * E},
      {"prod", k_pair_split<E, 4, 0, 2, false, 6623>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_BIG)
  // -DPB_SET_BIG: the multi-round regime (16384^2 / 32768^2 as one block, the
  // host launches without the wave priority): round-4 NP (7) against the
  // round-5 options without (6615) and with (6623) the priority, and subsets
  std::vector<Variant> vs = {
      {"opt7", k_pair_split<E, 4, 0, 2, false, 7>, 128, 4, 128 - 2 * E},
      {"opt6615", k_pair_split<E, 4, 0, 2, false, 6615>, 128, 4, 128 - 2 * E},
      {"opt6623", k_pair_split<E, 4, 0, 2, false, 6623>, 128, 4, 128 - 2 * E},
      {"opt2055", k_pair_split<E, 4, 0, 2, false, 2055>, 128, 4, 128 - 2 * E},
      {"opt87", k_pair_split<E, 4, 0, 2, false, 87>, 128, 4, 128 - 2 * E},
      {"opt343", k_pair_split<E, 4, 0, 2, false, 343>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_BIG2)
  // -DPB_SET_BIG2: the same regime, 343 (no period-aligned rings) with the tail
  // skip (128), the lattice-edge select (4096) and the priority (8) added
  std::vector<Variant> vs = {
      {"opt343", k_pair_split<E, 4, 0, 2, false, 343>, 128, 4, 128 - 2 * E},
      {"opt471", k_pair_split<E, 4, 0, 2, false, 471>, 128, 4, 128 - 2 * E},
      {"opt4439", k_pair_split<E, 4, 0, 2, false, 4439>, 128, 4, 128 - 2 * E},
      {"opt4567", k_pair_split<E, 4, 0, 2, false, 4567>, 128, 4, 128 - 2 * E},
      {"opt351", k_pair_split<E, 4, 0, 2, false, 351>, 128, 4, 128 - 2 * E},
      {"opt6615", k_pair_split<E, 4, 0, 2, false, 6615>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_PRIO)
  // -DPB_SET_PRIO: OPT 7 (before) against 15 (wave 1 at priority 3), interleaved
  std::vector<Variant> vs = {
      {"opt7", k_pair_split<E, 4, 0, 2, false, 7>, 128, 4, 128 - 2 * E},
      {"opt15", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt7_b", k_pair_split<E, 4, 0, 2, false, 7>, 128, 4, 128 - 2 * E},
      {"opt15_b", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"opt7_c", k_pair_split<E, 4, 0, 2, false, 7>, 128, 4, 128 - 2 * E},
      {"opt15_c", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
  };
#elif defined(PB_SET_DB)
  // -DPB_SET_DB: DMA depth / rows per barrier under the wave priority
  std::vector<Variant> vs = {
      {"D4_B2_o15", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"D8_B4_o15", k_pair_split<E, 8, 0, 4, false, 15>, 128, 4, 128 - 2 * E},
      {"D4_B4_o15", k_pair_split<E, 4, 0, 4, false, 15>, 128, 4, 128 - 2 * E},
      {"D6_B2_o15", k_pair_split<E, 6, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"D2_B2_o15", k_pair_split<E, 2, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"D4_B2_o15_b", k_pair_split<E, 4, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"D8_B4_o15_b", k_pair_split<E, 8, 0, 4, false, 15>, 128, 4, 128 - 2 * E},
      {"D4_B4_o15_b", k_pair_split<E, 4, 0, 4, false, 15>, 128, 4, 128 - 2 * E},
      {"D6_B2_o15_b", k_pair_split<E, 6, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
      {"D2_B2_o15_b", k_pair_split<E, 2, 0, 2, false, 15>, 128, 4, 128 - 2 * E},
  };
#else
  std::vector<Variant> vs = {
      {"D4_B2_opt1", k_pair_split<E, 4, 0, 2, false, 1>, 128, 4, 128 - 2 * E},
      {"D4_B2_opt5", k_pair_split<E, 4, 0, 2, false, 5>, 128, 4, 128 - 2 * E},
      {"D4_B2_opt7", k_pair_split<E, 4, 0, 2, false, 7>, 128, 4, 128 - 2 * E},
      {"D4_B2_opt1_b", k_pair_split<E, 4, 0, 2, false, 1>, 128, 4, 128 - 2 * E},
      {"D4_B2_opt5_b", k_pair_split<E, 4, 0, 2, false, 5>, 128, 4, 128 - 2 * E},
      {"D4_B2_opt7_b", k_pair_split<E, 4, 0, 2, false, 7>, 128, 4, 128 - 2 * E},
      {"D4_B2_opt1_c", k_pair_split<E, 4, 0, 2, false, 1>, 128, 4, 128 - 2 * E},
      {"D4_B2_opt5_c", k_pair_split<E, 4, 0, 2, false, 5>, 128, 4, 128 - 2 * E},
  };
#endif




  std::vector<double> ref((size_t)n * n), got((size_t)n * n);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // PB_REPS=R: the whole variant list R times over (interleaved A/B; the
  // first variant of the first round is the bitwise reference)
  const int reps = std::getenv("PB_REPS") ? std::max(1, std::atoi(std::getenv("PB_REPS"))) : 1;
  const size_t nv = vs.size();
  for (size_t vr = 0; vr < nv * (size_t)reps; ++vr) {
    const size_t vi = vr;
    const Variant &v = vs[vr % nv];
    // segment height: minimise rounds x (seg + 3E) over the resident slots
    const int nstrip = (int)ceil_div(n, v.strip_out);
    int seg = seg_force;
    if (!seg) {
      int64_t best = -1, bc = 0;
      for (int64_t k = 1; k <= 1024; ++k) {
        const int64_t sg = std::max<int64_t>(16, ceil_div(n, k));
        const int64_t wgs = nstrip * ceil_div(n, sg);
        const int64_t cost = ceil_div(wgs, (int64_t)v.wg_per_cu * cus) * (sg + 3 * E);
        if (best < 0 || cost < bc) {
          best = sg;
          bc = cost;
        }
        if (sg == 16) break;
      }
      seg = (int)best;
    }
    RectList L{};
    L.nrects = 1;
    Rect &R = L.r[0];
    R.pitch = pitch;
    R.x0 = 0;
    R.y0 = 0;
    R.x1 = n;
    R.y1 = n;
    R.gx0 = 0;
    R.gy0 = 0;
    R.seg_rows = seg;
    R.nstrip = nstrip;
    R.nseg = (int)ceil_div(n, seg);
    R.wg_begin = 0;
    L.nwork = R.nstrip * R.nseg;
    C.seg_pair = seg;
    // same initial field for every variant
    CK(hipMemcpy2D(origin(buf[0]), pitch * 8, h.data(), (size_t)n * 8, (size_t)n * 8, n, hipMemcpyHostToDevice));
    int cur = 0;
    auto launch = [&](int k) {
      R.u = origin(buf[cur]);
      R.un = origin(buf[1 - cur]);
      for (int j = 0; j < k; ++j) {
        L.r[0].u = origin(buf[cur]);
        L.r[0].un = origin(buf[1 - cur]);
        hipLaunchKernelGGL(v.fn, dim3(L.nwork), dim3(v.threads), 0, 0, L, C);
        cur = 1 - cur;
      }
    };
#if defined(PB_SET_TESTABL)
    // test mode: an L_h[W0] field in the block layout and the sin tables
    static double *lwb = nullptr, *dsx = nullptr, *dsy = nullptr;
    if (!lwb) {
      CK(hipMalloc(&lwb, bytes));
      CK(hipMemset(lwb, 0, bytes));
      std::vector<double> t(n + 4 * E);
      for (int g = 0; g < n + 4 * E; ++g) t[g] = std::sin(2 * M_PI * ((g - E) * dh));
      CK(hipMalloc(&dsx, t.size() * 8));
      CK(hipMalloc(&dsy, t.size() * 8));
      CK(hipMemcpy(dsx, t.data(), t.size() * 8, hipMemcpyHostToDevice));
      CK(hipMemcpy(dsy, t.data(), t.size() * 8, hipMemcpyHostToDevice));
    }
    // the separable L_h[W0] tables (nlh_device.h StepConst lsx / lty) and,
    // for the DMA variants, the same L_h[W0] field (long double, rounded)
    static double *dlsx = nullptr, *dlty = nullptr;
    if (!dlsx) {
      constexpr int NLV = pair_sep_nlv(E), LTS = pair_sep_stride(E);
      const int64_t ncol = pair_sep_ncol(E, n);
      auto sxe = [&](int64_t g) -> long double { return (g >= 0 && g < n) ? (long double)std::sin(2 * M_PI * (g * dh)) : 0.0L; };
      std::vector<double> lsx((NLV + 1) * ncol, 0.0), lty((size_t)(n + 4 * E) * LTS, 0.0);
      std::vector<long double> sxp((NLV + 1) * ncol, 0.0L), tyl((size_t)(n + 4 * E) * LTS, 0.0L);
      for (int64_t c = 0; c < ncol; ++c) {
        const int64_t g = c - 2 * E;
        if (g < 0 || g >= n) continue;
        for (int l = 0; l < NLV; ++l) {
          const int Lv = pair_sep_level(E, l);
          long double sum = 0.0L;
          for (int dx = -Lv; dx <= Lv; ++dx) sum += sxe(g + dx);
          sxp[l * ncol + c] = sum - (2 * Lv + 1) * sxe(g);
        }
        sxp[NLV * ncol + c] = sxe(g);
      }
      for (int64_t r = 0; r < n + 4 * E; ++r) {
        const int64_t y = r - 2 * E;
        if (y < 0 || y >= n) continue;
        for (int l = 0; l < NLV; ++l) {
          long double sum = 0.0L;
          for (int d = -E; d <= E; ++d)
            if (clen(E, d < 0 ? -d : d) == pair_sep_level(E, l)) sum += sxe(y + d);
          tyl[r * LTS + l] = sum;
        }
        long double z = -(long double)disk * sxe(y);
        for (int d = -E; d <= E; ++d) z += (2 * clen(E, d < 0 ? -d : d) + 1) * sxe(y + d);
        tyl[r * LTS + NLV] = z;
      }
      const long double cdl = (long double)C.c2d * (long double)C.dh2;  // folded into Sx' and sx
      for (size_t i = 0; i < lsx.size(); ++i) lsx[i] = (double)(sxp[i] * cdl);
      for (size_t i = 0; i < lty.size(); ++i) lty[i] = (double)tyl[i];
      CK(hipMalloc(&dlsx, lsx.size() * 8));
      CK(hipMalloc(&dlty, lty.size() * 8));
      CK(hipMemcpy(dlsx, lsx.data(), lsx.size() * 8, hipMemcpyHostToDevice));
      CK(hipMemcpy(dlty, lty.data(), lty.size() * 8, hipMemcpyHostToDevice));
      // the L_h[W0] field over the stage-1 rows / columns of every block row
      const long double cd = (long double)C.c2d * (long double)C.dh2;
      std::vector<double> lwh((size_t)pitch * rows, 0.0);
      for (int64_t y = -E; y < n + E; ++y)
        for (int64_t x = -E; x < n + E; ++x) {
          if (y < 0 || y >= n || x < 0 || x >= n) continue;
          long double v = sxp[NLV * ncol + x + 2 * E] * tyl[(y + 2 * E) * LTS + NLV];
          for (int l = 0; l < NLV; ++l) v += sxp[l * ncol + x + 2 * E] * tyl[(y + 2 * E) * LTS + l];
          lwh[(size_t)((y + H + kPairPadRows) * pitch + XL + x)] = (double)(cd * v);
        }
      CK(hipMemcpy(lwb, lwh.data(), lwh.size() * 8, hipMemcpyHostToDevice));
    }
    C.lsx = dlsx;
    C.lty = dlty;
    L.r[0].lw = origin(lwb);
    C.sxt = dsx;
    C.syt = dsy;
    C.st2pi = 0.1;
    C.ct = 0.9;
    C.st2pi2 = 0.11;
    C.ct2 = 0.89;
#endif
#if defined(PB_SET_TRACE)
    // every launch of an ABL 2048 variant writes its per-wave records through
    // Rc.lw: the buffer exists before the first launch (round 5: a launch with
    // lw still null faulted the GPU)
    uint64_t *dtr = nullptr;
    const size_t nrec = (size_t)L.nwork * 2 * 4;
    CK(hipMalloc(&dtr, nrec * 8));
    CK(hipMemset(dtr, 0, nrec * 8));
    L.r[0].lw = reinterpret_cast<const double *>(dtr);
    if (!L.r[0].lw) std::abort();
#endif
    launch(4);  // check pass count: identical for every variant
    CK(hipDeviceSynchronize());
    CK(hipMemcpy2D(got.data(), (size_t)n * 8, origin(buf[cur]), pitch * 8, (size_t)n * 8, n, hipMemcpyDeviceToHost));
    bool same = true;
    double maxd = 0;
    if (vi == 0) {
      ref = got;
    } else {
      same = std::memcmp(ref.data(), got.data(), ref.size() * 8) == 0;
      for (size_t i = 0; i < ref.size(); ++i) maxd = std::max(maxd, std::fabs(ref[i] - got[i]));
    }
#if defined(PB_SET_TRACE)
    {
      launch(20);
      CK(hipDeviceSynchronize());
      std::vector<uint64_t> tr(nrec);
      CK(hipMemcpy(tr.data(), dtr, nrec * 8, hipMemcpyDeviceToHost));
      const char *dir = std::getenv("PB_TRACE_DIR");
      std::string fn = std::string(dir ? dir : ".") + "/pair_trace_" + v.name + ".csv";
      FILE *f = std::fopen(fn.c_str(), "w");
      uint64_t t0 = ~0ull, t1 = 0, tmaxin = 0, tminout = ~0ull;
      double dsum = 0;
      int same_simd_role = 0, mixed = 0;
      std::vector<int> simd_role(8 * 64 * 4 * 4 * 2, 0);  // xcc, se*16+cu.. coarse key below
      if (f) std::fprintf(f, "block,wave,xcc,se,sh,cu,simd,wave_slot,t_entry,t_exit\n");
      // key (xcc, se, sh, cu, simd) -> roles seen
      std::vector<std::pair<uint64_t, int>> keys;
      for (int bidx = 0; bidx < L.nwork; ++bidx)
        for (int w = 0; w < 2; ++w) {
          const uint64_t *r = &tr[(size_t)(2 * bidx + w) * 4];
          const uint32_t hw = (uint32_t)r[0], xcc = (uint32_t)r[1] & 15;
          const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7,
                    ws = hw & 15;
          if (f) std::fprintf(f, "%d,%d,%u,%d,%d,%d,%d,%d,%llu,%llu\n", bidx, w, xcc, se, sh, cu, simd, ws,
                              (unsigned long long)r[2], (unsigned long long)r[3]);
          t0 = std::min(t0, r[2]);
          t1 = std::max(t1, r[3]);
          tmaxin = std::max(tmaxin, r[2]);
          tminout = std::min(tminout, r[3]);
          dsum += (double)(r[3] - r[2]);
          keys.push_back({((uint64_t)xcc << 20) | ((uint64_t)se << 12) | ((uint64_t)sh << 8) | ((uint64_t)cu << 4) |
                              (uint64_t)simd,
                          w});
        }
      if (f) std::fclose(f);
      std::sort(keys.begin(), keys.end());
      for (size_t a = 0; a < keys.size();) {
        size_t b2 = a;
        int n0 = 0, n1 = 0;
        while (b2 < keys.size() && keys[b2].first == keys[a].first) {
          (keys[b2].second ? n1 : n0)++;
          ++b2;
        }
        if (n0 && n1) ++mixed;
        else ++same_simd_role;
        a = b2;
      }
      // s_memrealtime ticks at 100 MHz
      std::printf("{\"trace\": \"%s\", \"wgs\": %d, \"span_us\": %.2f, \"last_entry_us\": %.2f, "
                  "\"first_exit_us\": %.2f, \"mean_wave_us\": %.2f, \"simds_mixed_roles\": %d, "
                  "\"simds_one_role\": %d}\n",
                  v.name, L.nwork, (t1 - t0) / 100.0, (tmaxin - t0) / 100.0, (tminout - t0) / 100.0,
                  dsum / (2.0 * L.nwork) / 100.0, mixed, same_simd_role);
      std::fflush(stdout);
    }
#endif
    launch(20);
    float best_ms = 1e30f;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0, 0));
      launch(passes);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best_ms = std::min(best_ms, ms);
    }
    const double us = best_ms * 1e3 / passes;
    std::printf("{\"rep\": %d, \"variant\": \"%s\", \"n\": %d, \"seg\": %d, \"wgs\": %d, \"us_per_pass\": %.2f, "
                "\"us_per_step\": %.2f, \"gnode_s\": %.1f, \"bitwise_vs_first\": %s, \"maxdiff\": %.3g}\n",
                (int)(vr / nv), v.name, n, seg, L.nwork, us, us / 2, 2.0 * n * n / us / 1e3, same ? "true" : "false", maxd);
    std::fflush(stdout);
#if defined(PB_SET_TRACE)
    CK(hipDeviceSynchronize());
    CK(hipFree(dtr));
#endif
  }
  return 0;
}
