// Device helpers shared by the MFMA GEMM kernels (gemm.hip, gemm_mx.hip).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "kernels.hpp"

// Row panels per tile-order group (tile_coords) when GemmParams.group is 0.
#ifndef CLIPGPU_TILE_GROUP
#define CLIPGPU_TILE_GROUP 8
#endif

namespace clipgpu {

// hipLaunchKernelGGL, or the event-stamped ext launch when a profiler armed g_gemm_events.
template <typename K, typename P>
inline void gemm_launch(K kernel, int grid, int threads, hipStream_t s, const P& p) {
  if (g_gemm_events.start && g_gemm_events.stop) {
    hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, g_gemm_events.start, g_gemm_events.stop, 0, p);
    g_gemm_events = GemmLaunchEvents();
  } else {
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, p);
  }
}

namespace gemm_detail {

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int N, typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}

template <int OFF, typename V>
__device__ __forceinline__ void ds_read_b128(V& r, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
}

template <int OFF, typename V>
__device__ __forceinline__ void ds_read_b64(V& r, uint32_t addr) {
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
}

// s_waitcnt lgkmcnt(0) that names every fragment register as read-write, so no
// consumer of them can be scheduled above it (cdna_hip_programming.md §5.7 form ii).
template <typename V, int MI, int NI>
__device__ __forceinline__ void lgkm_wait_all(V (&a)[MI], V (&b)[NI]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(a[i]));
#pragma unroll
  for (int i = 0; i < NI; ++i) asm volatile("" : "+v"(b[i]));
}

// Race-check builds only: NaN bytes over this lane's 16 bytes of an LDS-DMA destination (dst: the
// wave's 1 KiB piece), complete before the DMA is issued.  Inline asm on purpose: a plain C++ LDS
// store makes the compiler's wait insertion drain vmcnt first (it may alias the wave's pending
// LDS-DMAs), which would add exactly the synchronisation the race check exists to verify, and its
// extra live registers pushed a tile into spills once.
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_poison_piece(const char* dst) {
  const uint32_t a = lds_addr(dst) + (uint32_t)(threadIdx.x & 63) * 16u;
  const u32x4_t nan = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(a), "v"(nan) : "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}


// Tile order shared by all blocks: tiles are grouped `group` row panels at a time (walk M first
// inside a group) so that concurrently running tiles share A and W panels in L2.  group = 1 walks N
// first: the tiles of one row panel are neighbours, so one XCD's blocks read each A panel once and
// every XCD reads all of W (the order for a small W and a large A: c_proj).
__device__ __forceinline__ void tile_coords(int t, int nTm, int nTn, int BM, int BN, int& m0, int& n0,
                                            int group = CLIPGPU_TILE_GROUP) {
  const int per_group = group * nTn;
  const int first_m = (t / per_group) * group;
  const int gsize = min(nTm - first_m, group);
  m0 = (first_m + (t % per_group) % gsize) * BM;
  n0 = ((t % per_group) / gsize) * BN;
}

}  // namespace gemm_detail

}  // namespace clipgpu
