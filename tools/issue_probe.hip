// issue_probe.hip -- MI355X calibration of fp64 VALU issue throughput (tools
// only).  Each wave runs NACC independent chains of v_add_f64 (or v_fma_f64)
// for ITERS rounds; waves/SIMD is set by the grid (one 64-thread workgroup
// per wave, 256 CUs x 4 SIMDs).  Reports cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

template <int NACC, bool FMA>
__global__ __launch_bounds__(64) void chain(double *out, double a, double b, int iters) {
  double acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = threadIdx.x + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
      if (FMA)
        acc[k] = fma(acc[k], a, b);
      else
        acc[k] = acc[k] + a;
    }
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < NACC; ++k) s += acc[k];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int NACC, bool FMA>
static void run(double *out, int waves_per_simd) {
  const int iters = 4096;
  const int grid = 1024 * waves_per_simd;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  chain<NACC, FMA><<<grid, 64>>>(out, 1.0000001, 1e-9, iters);
  CK(hipEventRecord(e0));
  chain<NACC, FMA><<<grid, 64>>>(out, 1.0000001, 1e-9, iters);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double instr_per_simd = (double)iters * NACC * waves_per_simd;
  const double cyc = ms * 1e-3 * 2.4e9 / instr_per_simd;
  std::printf("{\"op\": \"%s\", \"nacc\": %d, \"waves_per_simd\": %d, \"us\": %.1f, "
              "\"cycles_per_instr_per_simd_at_2.4GHz\": %.2f}\n",
              FMA ? "v_fma_f64" : "v_add_f64", NACC, waves_per_simd, ms * 1e3, cyc);
}

int main() {
  double *out;
  CK(hipMalloc(&out, 1024 * 8 * 64 * sizeof(double)));
  for (int w : {1, 2, 4}) {
    run<1, false>(out, w);
    run<4, false>(out, w);
    run<8, false>(out, w);
    run<8, true>(out, w);
  }
  CK(hipFree(out));
  return 0;
}
