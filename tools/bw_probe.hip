// bw_probe.hip -- calibration of achievable HBM bandwidth for the stencil's
// access pattern on MI355X (tools only; not part of libnlh).
//
//   copy_vec   : un = u over the padded 4096^2 interior, 16 B per lane,
//                grid-stride (the guide's "float4 copy" ceiling)
//   strip_dma  : the fast kernel's memory structure with no arithmetic:
//                one wave per (strip, segment), rows streamed HBM -> LDS ring by
//                global_load_lds_dwordx4 D rows ahead, each row's 128 centre
//                values stored back from LDS
// Prints one JSON line per variant: time per launch and GB/s (16 B / node).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

constexpr int N = 4096, E = 8, XL = 8, PITCH = XL + N + XL + 112;  // 4224
constexpr int ROWS = N + 2 * E;

__device__ __forceinline__ void dma16(const void *g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(g), "s"(lds) : "memory");
}
template <int NN>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(NN) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

__global__ __launch_bounds__(256) void copy_vec(const double *__restrict__ u, double *__restrict__ un) {
  const int64_t n2 = (int64_t)N * N / 2;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n2; e += (int64_t)gridDim.x * 256) {
    const int64_t k = 2 * e;
    const int64_t y = k / N, x = k % N;
    const int64_t o = (y + E) * PITCH + XL + x;
    *reinterpret_cast<double2 *>(un + o) = *reinterpret_cast<const double2 *>(u + o);
  }
}

template <int D>
__global__ __launch_bounds__(64) void strip_dma(const double *__restrict__ u, double *__restrict__ un,
                                                int seg_h, int nstrip) {
  constexpr int RW = 128 + 16, K = D + 1;
  __shared__ __attribute__((aligned(16))) double ring[K * RW];
  const int lane = threadIdx.x;
  const int work = blockIdx.x;
  const int strip = work % nstrip, seg = work / nstrip;
  const int x0 = strip * 128, Y0 = seg * seg_h, Y1 = min(Y0 + seg_h, N);
  const int n_in = Y1 - Y0 + 2 * E;
  const double *g0 = u + (int64_t)(Y0) * PITCH + XL + x0 - 8;  // padded row Y0 - E + E
  const uint32_t lr = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  auto issue = [&](int i, int slot) {
    const int rr = min(i, n_in - 1);
    const double *g = g0 + (int64_t)rr * PITCH;
    dma16(g + 2 * lane, lr + slot * RW * 8);
    if (lane < 8) dma16(g + 128 + 2 * lane, lr + slot * RW * 8 + 1024);
  };
  for (int s = 0; s < D; ++s) issue(s, s);
  for (int i = 0; i < n_in; ++i) {
    issue(i + D, (i + D) % K);
    wait_vm<2 * D>();
    const double2 v = *reinterpret_cast<const double2 *>(&ring[(i % K) * RW + 8 + 2 * lane]);
    if (i >= 2 * E) {
      const int y = Y0 + i - 2 * E;
      *reinterpret_cast<double2 *>(un + (int64_t)(y + E) * PITCH + XL + x0 + 2 * lane) = v;
    }
  }
  wait_vm<0>();
}

// same, but the steady state waits with the exact in-order count: every
// older iteration also issued one store, so D*(2+1) ops are younger than the
// row being consumed (the warm-up rows, which store nothing, wait for 2*D)
template <int D>
__global__ __launch_bounds__(64) void strip_dma_x(const double *__restrict__ u, double *__restrict__ un,
                                                  int seg_h, int nstrip) {
  constexpr int RW = 128 + 16, K = D + 1;
  __shared__ __attribute__((aligned(16))) double ring[K * RW];
  const int lane = threadIdx.x;
  const int work = blockIdx.x;
  const int strip = work % nstrip, seg = work / nstrip;
  const int x0 = strip * 128, Y0 = seg * seg_h, Y1 = min(Y0 + seg_h, N);
  const int n_in = Y1 - Y0 + 2 * E;
  const double *g0 = u + (int64_t)(Y0) * PITCH + XL + x0 - 8;
  const uint32_t lr = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  auto issue = [&](int i, int slot) {
    const int rr = min(i, n_in - 1);
    const double *g = g0 + (int64_t)rr * PITCH;
    dma16(g + 2 * lane, lr + slot * RW * 8);
    if (lane < 8) dma16(g + 128 + 2 * lane, lr + slot * RW * 8 + 1024);
  };
  for (int s = 0; s < D; ++s) issue(s, s);
  int i = 0;
  for (; i < n_in && i < 2 * E + D; ++i) {
    issue(i + D, (i + D) % K);
    wait_vm<2 * D>();
    const double2 v = *reinterpret_cast<const double2 *>(&ring[(i % K) * RW + 8 + 2 * lane]);
    if (i >= 2 * E) {
      const int y = Y0 + i - 2 * E;
      *reinterpret_cast<double2 *>(un + (int64_t)(y + E) * PITCH + XL + x0 + 2 * lane) = v;
    }
  }
  for (; i < n_in; ++i) {
    issue(i + D, (i + D) % K);
    wait_vm<3 * D>();
    const double2 v = *reinterpret_cast<const double2 *>(&ring[(i % K) * RW + 8 + 2 * lane]);
    const int y = Y0 + i - 2 * E;
    *reinterpret_cast<double2 *>(un + (int64_t)(y + E) * PITCH + XL + x0 + 2 * lane) = v;
  }
  wait_vm<0>();
}

// strip/segment order, plain 16-B register loads (no LDS): isolates the
// access order from the LDS-DMA mechanism
template <int U>
__global__ __launch_bounds__(64) void strip_reg(const double *__restrict__ u, double *__restrict__ un,
                                                int seg_h, int nstrip) {
  const int lane = threadIdx.x;
  const int strip = blockIdx.x % nstrip, seg = blockIdx.x / nstrip;
  const int x0 = strip * 128, Y0 = seg * seg_h, Y1 = min(Y0 + seg_h, N);
  for (int y = Y0; y < Y1; y += U) {
    double2 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      v[k] = *reinterpret_cast<const double2 *>(u + (int64_t)(min(y + k, N - 1) + E) * PITCH + XL + x0 + 2 * lane);
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (y + k < Y1)
        *reinterpret_cast<double2 *>(un + (int64_t)(y + k + E) * PITCH + XL + x0 + 2 * lane) = v[k];
  }
}

// strip_dma variants: TAIL = also fetch the 16-double halo tail; NT = nt loads
template <int D, bool TAIL, bool NT>
__global__ __launch_bounds__(64) void strip_dma_v(const double *__restrict__ u, double *__restrict__ un,
                                                  int seg_h, int nstrip) {
  constexpr int RW = 128 + 16, K = D + 1;
  __shared__ __attribute__((aligned(16))) double ring[K * RW];
  const int lane = threadIdx.x;
  const int strip = blockIdx.x % nstrip, seg = blockIdx.x / nstrip;
  const int x0 = strip * 128, Y0 = seg * seg_h, Y1 = min(Y0 + seg_h, N);
  const int n_in = Y1 - Y0 + 2 * E;
  const double *g0 = u + (int64_t)(Y0) * PITCH + XL + x0 - 8;
  const uint32_t lr = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  auto issue = [&](int i, int slot) {
    const int rr = min(i, n_in - 1);
    const double *g = g0 + (int64_t)rr * PITCH;
    if (NT)
      asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off nt" : : "v"(g + 2 * lane), "s"(lr + slot * RW * 8) : "memory");
    else
      dma16(g + 2 * lane, lr + slot * RW * 8);
    if (TAIL && lane < 8) dma16(g + 128 + 2 * lane, lr + slot * RW * 8 + 1024);
  };
  constexpr int G = TAIL ? 2 : 1;
  for (int s = 0; s < D; ++s) issue(s, s);
  for (int i = 0; i < n_in; ++i) {
    issue(i + D, (i + D) % K);
    wait_vm<G * D>();
    const double2 v = *reinterpret_cast<const double2 *>(&ring[(i % K) * RW + 8 + 2 * lane]);
    if (i >= 2 * E) {
      const int y = Y0 + i - 2 * E;
      *reinterpret_cast<double2 *>(un + (int64_t)(y + E) * PITCH + XL + x0 + 2 * lane) = v;
    }
  }
  wait_vm<0>();
}

// random (non-zero, full-entropy mantissa) doubles: HBM power and so
// throughput depends on the data toggled, a memset-0 buffer flatters a probe
__global__ void fill_random(double *u, int64_t n) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    uint64_t z = (uint64_t)e * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    u[e] = (double)(z >> 11) * 0x1.0p-53 - 0.5;
  }
}

template <class F>
static float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) f();
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char **argv) {
  const bool full = argc > 1 && std::string(argv[1]) == "--full";
  const size_t bytes = (size_t)PITCH * ROWS * sizeof(double);
  double *u, *un;
  CK(hipMalloc(&u, bytes));
  CK(hipMalloc(&un, bytes));
  const double algo = 16.0 * N * N;
  const int nstrip = N / 128;
  for (int data = 0; data < 2; ++data) {
    const char *dn = data ? "random" : "zero";
    if (data) {
      fill_random<<<4096, 256>>>(u, (int64_t)bytes / 8);
      fill_random<<<4096, 256>>>(un, (int64_t)bytes / 8);
    } else {
      CK(hipMemset(u, 0, bytes));
      CK(hipMemset(un, 0, bytes));
    }
    CK(hipDeviceSynchronize());
    for (int g : {1024, 8192}) {
      const float ms = time_it([&] { copy_vec<<<g, 256>>>(u, un); }, 50);
      std::printf("{\"data\": \"%s\", \"variant\": \"copy_vec\", \"grid\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
                  dn, g, ms * 1e3, algo / (ms * 1e-3) / 1e9);
    }
    for (int seg : {64, 128, 256}) {
      const int nseg = (N + seg - 1) / seg;
      float c = time_it([&] { strip_dma_v<8, true, false><<<nstrip * nseg, 64>>>(u, un, seg, nstrip); }, 50);
      float e = time_it([&] { strip_dma_v<8, true, true><<<nstrip * nseg, 64>>>(u, un, seg, nstrip); }, 50);
      std::printf("{\"data\": \"%s\", \"variant\": \"strip_dma\", \"seg\": %d, \"wgs\": %d, "
                  "\"dma_tail\": %.2f, \"dma_tail_nt\": %.2f}\n", dn, seg, nstrip * nseg, c * 1e3, e * 1e3);
    }
    if (!full) continue;
    for (int seg : {32, 64, 128, 256}) {
      const int nseg = (N + seg - 1) / seg;
      float ms4 = time_it([&] { strip_dma_x<4><<<nstrip * nseg, 64>>>(u, un, seg, nstrip); }, 50);
      float ms8 = time_it([&] { strip_dma_x<8><<<nstrip * nseg, 64>>>(u, un, seg, nstrip); }, 50);
      float a = time_it([&] { strip_reg<4><<<nstrip * nseg, 64>>>(u, un, seg, nstrip); }, 50);
      float d = time_it([&] { strip_dma_v<8, false, false><<<nstrip * nseg, 64>>>(u, un, seg, nstrip); }, 50);
      std::printf("{\"data\": \"%s\", \"variant\": \"detail\", \"seg\": %d, \"exactwait_D4\": %.2f, "
                  "\"exactwait_D8\": %.2f, \"reg_U4\": %.2f, \"dma_notail\": %.2f}\n",
                  dn, seg, ms4 * 1e3, ms8 * 1e3, a * 1e3, d * 1e3);
    }
  }
  CK(hipFree(u));
  CK(hipFree(un));
  return 0;
}
