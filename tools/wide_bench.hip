// wide_bench.hip -- standalone timing harness: single-step large-horizon
// kernels (k_fast R=1 vs k_wide variants, nlh_wide.h) on one C4-sized block
// (8192^2, eps=32).  Results compared with the first variant within the fast
// kernels' tolerance (different summation order).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Inonlocalheatequation_amd/csrc \
//     -mllvm -pragma-unroll-threshold=1000000 tools/wide_bench.hip -o build/wide_bench
//   build/wide_bench [n=8192] [steps=20]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nlh_fast.h"
#include "nlh_wide.h"

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
  int strip;      // output columns per strip
  int wg_per_cu;  // resident workgroups per CU
  int threads = 64;  // 64 x waves per workgroup
};

#ifndef WB_E
#define WB_E 32
#endif
constexpr int E = WB_E;  // -DWB_E=56: the compile-time instance of another horizon
static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 8192;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 20;
  const int H = E, XL = E > 32 ? (E + 7) / 8 * 8 : 32;  // staged rows start EP columns left of a strip
  const int64_t pitch = (XL + ceil_div(n, 256) * 256 + XL + 7) / 8 * 8;
  const int64_t rows = n + 2 * H;
  const size_t bytes = (size_t)(pitch * rows) * sizeof(double) + 256;
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
  // variants: prefix-sum rows (production, PA = 0) and prefix rows built PA
  // rows ahead (k_wide PA), at DMA depths 6 and 8
#if WB_E <= 32
  // production form (prefix rows two ahead, interleaved scan, row pairs) with
  // the per-store row multiply vs the chunk's row pointer (SP)
#define KW(SP) k_wide<E, 8, false, 6, 0, 1, false, 16, true, true, 2, true, true, true, true, SP>
  std::vector<Variant> vs = {
      {"prod", KW(false), 64, 8, 64},
      {"sp", KW(true), 64, 8, 64},
      {"prod_b", KW(false), 64, 8, 64},
      {"sp_b", KW(true), 64, 8, 64},
      {"prod_c", KW(false), 64, 8, 64},
      {"sp_c", KW(true), 64, 8, 64},
  };
#else
  // nested windows, 8-row chunks (the production form past eps 35), one row
  // at a time vs row pairs; one wave per SIMD past eps 40 (AGPRs)
  std::vector<Variant> vs = {
      {"nested_C8_D6", k_wide<E, 8, false, 6>, 64, 4},
      {"nested_C8_D6_rp", k_wide<E, 8, false, 6, 0, 1, false, 16, true, false, 0, false, false, false, true>, 64, 4},
      {"nested_C8_D6_rp_sp", k_wide<E, 8, false, 6, 0, 1, false, 16, true, false, 0, false, false, false, true, true>,
       64, 4},
      {"nested_C8_D6_rp_b", k_wide<E, 8, false, 6, 0, 1, false, 16, true, false, 0, false, false, false, true>, 64, 4},
      {"nested_C8_D6_rp_sp_b", k_wide<E, 8, false, 6, 0, 1, false, 16, true, false, 0, false, false, false, true, true>,
       64, 4},
  };
#endif

  std::vector<double> ref((size_t)n * n), got((size_t)n * n);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (size_t vi = 0; vi < vs.size(); ++vi) {
    const Variant &v = vs[vi];
    const int nstrip = (int)ceil_div(n, v.strip);
    const int64_t slots = (int64_t)v.wg_per_cu * cus;
    const int seg = (int)std::max<int64_t>(2 * E, ceil_div((int64_t)nstrip * n, slots));
    RectList L{};
    L.nrects = 1;
    Rect &R = L.r[0];
    R.pitch = pitch;
    R.x1 = n;
    R.y1 = n;
    R.seg_rows = seg;
    R.nstrip = nstrip;
    R.nseg = (int)ceil_div(n, seg);
    L.nwork = R.nstrip * R.nseg;
    C.seg_h = seg;
    CK(hipMemcpy2D(origin(buf[0]), pitch * 8, h.data(), (size_t)n * 8, (size_t)n * 8, n, hipMemcpyHostToDevice));
    int cur = 0;
    auto launch = [&](int k) {
      for (int j = 0; j < k; ++j) {
        L.r[0].u = origin(buf[cur]);
        L.r[0].un = origin(buf[1 - cur]);
        hipLaunchKernelGGL(v.fn, dim3(L.nwork), dim3(v.threads), 0, 0, L, C);
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
    launch(2);
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
    std::printf("{\"variant\": \"%s\", \"n\": %d, \"seg\": %d, \"wgs\": %d, \"us_per_step\": %.1f, "
                "\"gnode_s\": %.1f, \"maxdiff_rel\": %.3g}\n",
                v.name, n, seg, L.nwork, us, (double)n * n / us / 1e3, maxd / scale);
    std::fflush(stdout);
  }
  return 0;
}
