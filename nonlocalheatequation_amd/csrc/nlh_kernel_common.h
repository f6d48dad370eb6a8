// nlh_kernel_common.h -- device helpers shared by the gfx950 kernels
// (nlh_kernels.hip, nlh_fast.h instantiation units).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "nlh_device.h"

namespace nlh {

// ----------------------------------------------------------------------------
// helpers

// XCD-aware bijective remap: hardware deals workgroup ids round-robin over
// the 8 XCDs; give each XCD a contiguous range of work items so that strips
// sharing halo columns / warm-up rows hit the same L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7, l = bid >> 3;
  return (x < r) ? x * (q + 1) + l : r * (q + 1) + (x - r) * q + l;
}

__device__ __forceinline__ int find_rect(const RectList &L, int work) {
  int ri = 0;
  for (int k = 1; k < L.nrects; ++k) ri = (work >= L.r[k].wg_begin) ? k : ri;
  return ri;
}

// floor(sqrt(E^2 - d^2)) == (long)sqrt((double)(E*E - d*d)) of the
// reference's len_1d_line (:231) for every integer argument < 2^52.
__host__ __device__ constexpr int clen(int E, int d) {
  int L = 0;
  while ((L + 1) * (L + 1) <= E * E - d * d) ++L;
  return L;
}

__host__ __device__ constexpr int pow2_ceil(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

__host__ __device__ constexpr int disk_count(int E) {
  int n = 0;
  for (int d = -E; d <= E; ++d) n += 2 * clen(E, d < 0 ? -d : d) + 1;
  return n;
}

// One 16-byte-per-lane LDS-DMA: LDS[lds + 16*lane] <- global[g].  `nt`
// (non-temporal): the field is streamed once per step; on MI355X the
// stencil's DMA skeleton runs 48.3 -> 39.4 us with it (profiles/r01/bw_probe_v3.txt).
__device__ __forceinline__ void dma16(const void *g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off nt"
               :
               : "v"(g), "s"(lds)
               : "memory");
}

__device__ __forceinline__ void dma16_plain(const void *g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(g), "s"(lds)
               : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(N) : "memory");
}

// NCH 16-byte chunks starting at g -> LDS starting at lds.
// NTF / NTP: non-temporal hint on the full 64-lane chunks / the partial tail
template <int NCH, bool NTF = true, bool NTP = true>
__device__ __forceinline__ void dma_chunks(const double *g, uint32_t lds,
                                           int lane) {
#pragma unroll
  for (int k = 0; k < (NCH + 63) / 64; ++k) {
    const double *src = g + 2 * (k * 64 + lane);
    if (k * 64 + 64 <= NCH) {
      if (NTF) dma16(src, lds + k * 1024); else dma16_plain(src, lds + k * 1024);
    } else if (lane < NCH - k * 64) {
      if (NTP) dma16(src, lds + k * 1024); else dma16_plain(src, lds + k * 1024);
    }
  }
}

// f(integral_constant<int, I>) for I = 0 .. N-1, fully unrolled
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F &&f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

}  // namespace nlh
