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
#if defined(PB_SET_PRIO)
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
  for (size_t vi = 0; vi < vs.size(); ++vi) {
    const Variant &v = vs[vi];
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
    std::printf("{\"variant\": \"%s\", \"n\": %d, \"seg\": %d, \"wgs\": %d, \"us_per_pass\": %.2f, "
                "\"us_per_step\": %.2f, \"gnode_s\": %.1f, \"bitwise_vs_first\": %s, \"maxdiff\": %.3g}\n",
                v.name, n, seg, L.nwork, us, us / 2, 2.0 * n * n / us / 1e3, same ? "true" : "false", maxd);
    std::fflush(stdout);
  }
  return 0;
}
