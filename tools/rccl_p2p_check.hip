// rccl_p2p_check.hip -- standalone RCCL point-to-point check, no libnlh
// (VERDICT r4, next 4).  One process, a one-rank communicator
// (ncclGetUniqueId + ncclCommInitRank(1)), send/recv to self inside one
// group on a non-blocking stream, as libnlh's virtual-rank tile moves post
// them (nlh_api.cpp, nlh_repartition).  For each message size the send buffer
// holds a per-element pattern, the receive buffer a sentinel; a device
// kernel then checks every element and reports the mismatches and the first
// and last bad element.  "chunks" > 1 posts the same bytes as that many
// in-order messages (libnlh's kP2PChunk = 256 MiB form).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/rccl_p2p_check.hip \
//     -o build/rccl_p2p_check -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
//   build/rccl_p2p_check [max_gib=3]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)
#define NK(x)                                                                                   \
  do {                                                                                          \
    ncclResult_t r_ = (x);                                                                      \
    if (r_ != ncclSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_));   \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

__device__ __forceinline__ uint64_t pattern(uint64_t i, uint64_t salt) {
  uint64_t z = i + salt * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_fill(uint64_t *p, size_t n, uint64_t salt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = salt == 0 ? 0xDEADBEEFDEADBEEFull : pattern(i, salt);
}

// out[0] = mismatches, out[1] = first bad index, out[2] = last bad index
__global__ void k_check(const uint64_t *p, size_t n, uint64_t salt, unsigned long long *out) {
  unsigned long long bad = 0, lo = ~0ull, hi = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (p[i] != pattern(i, salt)) {
      ++bad;
      lo = std::min<unsigned long long>(lo, i);
      hi = std::max<unsigned long long>(hi, i);
    }
  if (bad) {
    atomicAdd(&out[0], bad);
    atomicMin(&out[1], lo);
    atomicMax(&out[2], hi);
  }
}

int main(int argc, char **argv) {
  const double max_gib = argc > 1 ? std::atof(argv[1]) : 3.0;
  int ver = 0;
  NK(ncclGetVersion(&ver));
  const size_t max_n = (size_t)(max_gib * (1ull << 30)) / 8;
  uint64_t *sb = nullptr, *rb = nullptr;
  unsigned long long *dout = nullptr;
  CK(hipMalloc(&sb, max_n * 8));
  CK(hipMalloc(&rb, max_n * 8));
  CK(hipMalloc(&dout, 3 * sizeof(unsigned long long)));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  ncclUniqueId id;
  NK(ncclGetUniqueId(&id));
  ncclComm_t comm;
  NK(ncclCommInitRank(&comm, 1, id, 0));

  struct Case {
    double gib;
    int chunks;
    bool dbl;  // ncclDouble (libnlh's type) or ncclUint8
  };
  std::vector<Case> cases = {{0.5, 1, true},  {1.0, 1, true},  {1.25, 1, true}, {1.5, 1, true},
                             {2.0, 1, true},  {2.5, 1, true},  {3.0, 1, true},  {1.5, 1, false},
                             {3.0, 1, false}, {1.5, 6, true},  {3.0, 12, true}, {1.5, 1, true}};
  int failures = 0;
  uint64_t salt = 1;
  for (const Case &c : cases) {
    if (c.gib > max_gib + 1e-9) continue;
    const size_t n = (size_t)(c.gib * (1ull << 30)) / 8;
    ++salt;
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, st, sb, n, salt);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, st, rb, n, (uint64_t)0);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(st));
    NK(ncclGroupStart());
    const size_t per = (n + c.chunks - 1) / c.chunks;
    for (size_t o = 0; o < n; o += per) {
      const size_t m = std::min(per, n - o);
      if (c.dbl) {
        NK(ncclSend(sb + o, m, ncclDouble, 0, comm, st));
        NK(ncclRecv(rb + o, m, ncclDouble, 0, comm, st));
      } else {
        NK(ncclSend(sb + o, m * 8, ncclUint8, 0, comm, st));
        NK(ncclRecv(rb + o, m * 8, ncclUint8, 0, comm, st));
      }
    }
    NK(ncclGroupEnd());
    CK(hipStreamSynchronize(st));
    unsigned long long init[3] = {0, ~0ull, 0}, res[3];
    CK(hipMemcpy(dout, init, sizeof(init), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, st, rb, n, salt, dout);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(res, dout, sizeof(res), hipMemcpyDeviceToHost));
    const bool ok = res[0] == 0;
    failures += !ok;
    std::printf("{\"rccl_version\": %d, \"gib\": %.2f, \"elements\": %zu, \"type\": \"%s\", \"chunks\": %d, "
                "\"bad_elements\": %llu, \"first_bad\": %lld, \"last_bad\": %lld, \"ok\": %s}\n",
                ver, c.gib, n, c.dbl ? "double" : "uint8", c.chunks, res[0], ok ? -1ll : (long long)res[1],
                ok ? -1ll : (long long)res[2], ok ? "true" : "false");
    std::fflush(stdout);
  }
  ncclCommDestroy(comm);
  CK(hipFree(sb));
  CK(hipFree(rb));
  std::printf("{\"summary\": \"%s\", \"failed_cases\": %d}\n", failures ? "corruption reproduced" : "all whole",
              failures);
  return 0;
}
