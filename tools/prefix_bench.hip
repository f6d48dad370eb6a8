// prefix_bench.hip -- standalone timing harness of k_prefix_rt (nlh_prefix.h)
// on one C4-sized block (n^2, production step) at run-time horizons, with
// variants of its template knobs (rows per work item R, SKIP).  Results are
// compared with the first variant (same sums; SKIP and R change nothing but
// which zero pairs are added, so the fields are bitwise equal).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Inonlocalheatequation_amd/csrc \
//     tools/prefix_bench.hip nonlocalheatequation_amd/csrc/nlh_prefix.hip -o build/prefix_bench
//   build/prefix_bench [n=8192] [steps=10] E...
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nlh_prefix.h"

using namespace nlh;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef void (*KFn)(RectList, StepConst, const int2 *);
struct Variant {
  const char *name;
  KFn fn;
  int rows;  // R
  int cpl = 1;  // columns per lane
};

static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

static std::vector<int32_t> table(int E, int R) {
  std::vector<int32_t> t(2 * (2 * (E + R) + 1));
  for (int i = 0; i < 2 * (E + R) + 1; ++i) {
    const int d = i - E - R, ad = d < 0 ? -d : d;
    const int L = ad <= E ? clen(E, ad) : 0;
    t[2 * i] = ad <= E ? L : 0;
    t[2 * i + 1] = ad <= E ? -L - 1 : 0;
  }
  return t;
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 8192;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 10;
  std::vector<int> eps;
  for (int i = 3; i < argc; ++i) eps.push_back(std::atoi(argv[i]));
  if (eps.empty()) eps = {48, 64, 80, 96};
  // round 4 (profiles/r04/first/prefix_bench.jsonl): R = 32 without SKIP /
  // RUN was the fastest everywhere (the uniform branches serialise the LDS
  // reads; R 48 / 64 cost occupancy)
#if defined(PX_SET_PEEL)
  // -DPX_SET_PEEL: round 5, the partial-horizon rows peeled (PEEL) against the round-4 form
  std::vector<Variant> vs4 = {
      {"R32", k_prefix_rt<4, 32, false>, 32},
      {"R32_peel", k_prefix_rt<4, 32, false, false, false, 1, true>, 32},
      {"R32_b", k_prefix_rt<4, 32, false>, 32},
      {"R32_peel_b", k_prefix_rt<4, 32, false, false, false, 1, true>, 32},
  };
  std::vector<Variant> vs6 = {
      {"NV6_R32", k_prefix_rt<6, 32, false>, 32},
      {"NV6_R32_peel", k_prefix_rt<6, 32, false, false, false, 1, true>, 32},
  };
  std::vector<Variant> vs8 = {
      {"NV8_R32", k_prefix_rt<8, 32, false>, 32},
      {"NV8_R32_peel", k_prefix_rt<8, 32, false, false, false, 1, true>, 32},
  };
#else
  std::vector<Variant> vs4 = {
      {"R32", k_prefix_rt<4, 32, false>, 32},
      {"R32_cpl2_nv6", k_prefix_rt<6, 32, false, false, false, 2>, 32, 2},
      {"R16_cpl2_nv6", k_prefix_rt<6, 16, false, false, false, 2>, 16, 2},
      {"R24_cpl2_nv6", k_prefix_rt<6, 24, false, false, false, 2>, 24, 2},
  };

  std::vector<Variant> vs6 = {
      {"NV6_R32", k_prefix_rt<6, 32, false>, 32},
      {"R32_cpl2_nv8", k_prefix_rt<8, 32, false, false, false, 2>, 32, 2},
      {"R16_cpl2_nv8", k_prefix_rt<8, 16, false, false, false, 2>, 16, 2},
  };
  std::vector<Variant> vs8 = {
      {"R32", k_prefix_rt<8, 32, false, false>, 32},
      {"R32_skip", k_prefix_rt<8, 32, false, true>, 32},
      {"R48_skip", k_prefix_rt<8, 48, false, true>, 48},
      {"R32_run", k_prefix_rt<8, 32, false, false, true>, 32},
      {"R48_run", k_prefix_rt<8, 48, false, false, true>, 48},
  };
#endif
  for (int E : eps) {
    const int H = E, XL = (E + 7) / 8 * 8;
    const int64_t pitch = (XL + ceil_div(n, 64) * 64 + 512 + 7) / 8 * 8;
    const int64_t rows = n + 2 * H;
    const size_t bytes = (size_t)(pitch * rows) * sizeof(double) + 4096;
    double *buf[2];
    for (auto &b : buf) {
      CK(hipMalloc(&b, bytes));
      CK(hipMemset(b, 0, bytes));
    }
    std::vector<double> h((size_t)n * n);
    const double dh = 1.0 / n;
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x)
        h[(size_t)y * n + x] = std::sin(2 * M_PI * (x * dh)) * std::sin(2 * M_PI * (y * dh)) +
                               0.25 * std::sin(2 * M_PI * (7 * x * dh + 3 * y * dh));
    auto origin = [&](double *b) { return b + (int64_t)H * pitch + XL; };
    const int disk = disk_count(E);
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
    std::vector<double> ref((size_t)n * n), got((size_t)n * n);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const auto &vs = E <= 96 ? vs4 : E <= 160 ? vs6 : vs8;
    for (size_t vi = 0; vi < vs.size(); ++vi) {
      const Variant &v = vs[vi];
      const std::vector<int32_t> tab = table(E, v.rows);
      int32_t *dtab = nullptr;
      CK(hipMalloc(&dtab, tab.size() * 4));
      CK(hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
      RectList L{};
      L.nrects = 1;
      Rect &R = L.r[0];
      R.pitch = pitch;
      R.x1 = n;
      R.y1 = n;
      R.seg_rows = v.rows;
      R.nstrip = (int)ceil_div(n, 64 * v.cpl);
      R.nseg = (int)ceil_div(n, v.rows);
      L.nwork = R.nstrip * R.nseg;
      CK(hipMemcpy2D(origin(buf[0]), pitch * 8, h.data(), (size_t)n * 8, (size_t)n * 8, n, hipMemcpyHostToDevice));
      int cur = 0;
      auto launch = [&](int k) {
        for (int j = 0; j < k; ++j) {
          L.r[0].u = origin(buf[cur]);
          L.r[0].un = origin(buf[1 - cur]);
          hipLaunchKernelGGL(v.fn, dim3(L.nwork), dim3(64), 0, 0, L, C, (const int2 *)dtab);
          cur = 1 - cur;
        }
      };
      launch(2);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy2D(got.data(), (size_t)n * 8, origin(buf[cur]), pitch * 8, (size_t)n * 8, n, hipMemcpyDeviceToHost));
      double maxd = 0, scale = 0;
      if (vi == 0) ref = got;
      for (size_t i = 0; i < ref.size(); ++i) {
        maxd = std::max(maxd, std::fabs(ref[i] - got[i]));
        scale = std::max(scale, std::fabs(ref[i]));
      }
      float best = 1e30f;
      for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0, 0));
        launch(steps);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms);
      }
      const double us = best * 1e3 / steps;
      std::printf("{\"variant\": \"%s\", \"eps\": %d, \"n\": %d, \"wgs\": %d, \"us_per_step\": %.1f, "
                  "\"gnode_s\": %.2f, \"maxdiff_rel\": %.3g}\n",
                  v.name, E, n, L.nwork, us, (double)n * n / us / 1e3, maxd / scale);
      std::fflush(stdout);
      CK(hipFree(dtab));
    }
    for (auto &b : buf) CK(hipFree(b));
  }
  return 0;
}
