// Probe: how long does the hardware take to start every block of a one-round launch, by block
// shape?  The round-3 stamps of the table GEMM tiles showed block start times spread over 4-5 µs
// (480 blocks of 512 threads, 75 KiB LDS, 128 VGPRs) where the guide quotes 0.34-0.69 µs for a
// 1024-block grid.  Each variant stamps s_memrealtime (100 MHz, chip-wide) at block entry, then
// holds its CU for HOLD µs so that no block retires before the last one starts; prints the spread
// of start times.  Standalone: hipcc --offload-arch=gfx950 -O3 -o tools/bin/dispatch_probe
// tools/dispatch_probe.hip && tools/bin/dispatch_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr int HOLD_TICKS = 3000;  // 30 µs at 100 MHz

// VG: VGPRs the kernel is made to allocate (an asm clobber list), LDS: dynamic bytes asked.
template <int VG>
__global__ void probe(unsigned long long* out, int touch_lds) {
  extern __shared__ char lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (VG >= 128) asm volatile("" ::: "v0", "v8", "v16", "v24", "v32", "v40", "v48", "v56", "v64", "v72", "v80",
                                    "v88", "v96", "v104", "v112", "v120", "v127");
  if (VG >= 256) asm volatile("" ::: "v128", "v136", "v144", "v152", "v160", "v168", "v176", "v184", "v192",
                                    "v200", "v208", "v216", "v224", "v232", "v240", "v248", "v255");
  if (touch_lds) lds[threadIdx.x] = (char)threadIdx.x;
  if (threadIdx.x == 0) out[blockIdx.x] = t0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < HOLD_TICKS) __builtin_amdgcn_s_sleep(8);
}

// The GEMM's shape of entry: a 128-byte parameter struct by value (GemmParams-sized).  t0 at entry,
// t1 once the struct's values have arrived (they feed the stored value), so t1 - t0 is the
// kernel-argument fetch as the GEMM's prologue sees it.
struct Args {
  unsigned long long* out;
  long a[14];
  int n;
};
__global__ void probe_args(Args p) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  long acc = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) acc += p.a[i];
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  asm volatile("" : "+s"(t1) : "s"(acc));
  if (threadIdx.x == 0) {
    p.out[2 * blockIdx.x] = t0;
    p.out[2 * blockIdx.x + 1] = t1 + (acc == 12345 ? 1 : 0);
  }
  while (__builtin_amdgcn_s_memrealtime() - t0 < HOLD_TICKS) __builtin_amdgcn_s_sleep(8);
}

int run_args(int blocks, int threads, unsigned long long* d, std::vector<unsigned long long>& h) {
  Args a{};
  a.out = d;
  for (int i = 0; i < 14; ++i) a.a[i] = i;
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipMemset(d, 0, blocks * 16));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(probe_args, dim3(blocks), dim3(threads), 0, nullptr, a);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, blocks * 16, hipMemcpyDeviceToHost));
    unsigned long long mn = ~0ull;
    for (int i = 0; i < blocks; ++i) mn = std::min(mn, h[2 * i]);
    std::vector<double> s0(blocks), s1(blocks), dl(blocks);
    for (int i = 0; i < blocks; ++i) {
      s0[i] = (h[2 * i] - mn) / 100.0;
      s1[i] = (h[2 * i + 1] - mn) / 100.0;
      dl[i] = (double)(h[2 * i + 1] - h[2 * i]) / 100.0;
    }
    std::sort(s0.begin(), s0.end());
    std::sort(s1.begin(), s1.end());
    std::sort(dl.begin(), dl.end());
    if (rep > 0)
      printf("128-B struct arg, %4d x %4d thr: entry spread p50 %.2f max %.2f | after-args spread p50 %.2f max %.2f | "
             "arg fetch p50 %.2f max %.2f us\n", blocks, threads, s0[blocks / 2], s0[blocks - 1], s1[blocks / 2],
             s1[blocks - 1], dl[blocks / 2], dl[blocks - 1]);
  }
  return 0;
}

// A straight-line preamble of NI 4-byte VALU instructions between two stamps: t1 - t0 is what a
// cold (first launch) or warm (repeat launch) instruction cache costs for NI * 4 bytes of code.
#define PRE_16 "v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n" \
               "v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n" \
               "v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n" \
               "v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n v_add_u32_e32 v1, v1, v2\n"
#define PRE_128 PRE_16 PRE_16 PRE_16 PRE_16 PRE_16 PRE_16 PRE_16 PRE_16
template <int REPS128>
__global__ void probe_pre(unsigned long long* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int r = 0; r < REPS128; ++r) asm volatile(PRE_128 ::: "v1", "v2");
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t0;
    out[2 * blockIdx.x + 1] = t1;
  }
  while (__builtin_amdgcn_s_memrealtime() - t0 < HOLD_TICKS) __builtin_amdgcn_s_sleep(8);
}

template <int REPS128>
int run_pre(int blocks, int threads, unsigned long long* d, std::vector<unsigned long long>& h) {
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemset(d, 0, blocks * 16));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(probe_pre<REPS128>, dim3(blocks), dim3(threads), 0, nullptr, d);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, blocks * 16, hipMemcpyDeviceToHost));
    std::vector<double> dl(blocks);
    for (int i = 0; i < blocks; ++i) dl[i] = (double)(h[2 * i + 1] - h[2 * i]) / 100.0;
    std::sort(dl.begin(), dl.end());
    printf("preamble of %4d VALU instrs (%5d B), %4d x %4d thr, launch %d (%s): t1 - t0 p50 %.2f max %.2f us\n",
           REPS128 * 128, REPS128 * 512, blocks, threads, rep, rep == 0 ? "cold" : "repeat", dl[blocks / 2],
           dl[blocks - 1]);
  }
  return 0;
}

template <int VG>
int run(const char* name, int blocks, int threads, int lds, unsigned long long* d, std::vector<unsigned long long>& h) {
  if (lds > 65536) CK(hipFuncSetAttribute((const void*)probe<VG>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipMemset(d, 0, blocks * 8));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(probe<VG>, dim3(blocks), dim3(threads), lds, nullptr, d, 1);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, blocks * 8, hipMemcpyDeviceToHost));
    std::vector<double> s(blocks);
    const unsigned long long mn = *std::min_element(h.begin(), h.begin() + blocks);
    for (int i = 0; i < blocks; ++i) s[i] = (h[i] - mn) / 100.0;
    std::sort(s.begin(), s.end());
    if (rep > 0)
      printf("%-44s blocks %4d x %4d thr, LDS %6d, VGPR>=%3d: start spread p50 %.2f p90 %.2f max %.2f us\n", name,
             blocks, threads, lds, VG, s[blocks / 2], s[blocks * 9 / 10], s[blocks - 1]);
  }
  return 0;
}

int main() {
  unsigned long long* d;
  std::vector<unsigned long long> h(8192);
  CK(hipMalloc(&d, 8192 * 8));
  int rc = 0;
  rc |= run<0>("guide shape: 1024 x 256, no LDS", 1024, 256, 0, d, h);
  rc |= run<0>("480 x 512, no LDS", 480, 512, 0, d, h);
  rc |= run<0>("480 x 512, 75 KiB LDS (two per CU)", 480, 512, 76800, d, h);
  rc |= run<128>("480 x 512, 128 VGPR, no LDS", 480, 512, 0, d, h);
  rc |= run<128>("480 x 512, 128 VGPR, 75 KiB LDS (tile 17)", 480, 512, 76800, d, h);
  rc |= run<256>("256 x 512, 256 VGPR, 130 KiB LDS (tile 18)", 256, 512, 133120, d, h);
  rc |= run<0>("256 x 512, no LDS", 256, 512, 0, d, h);
  rc |= run<0>("3072 x 256, 18 KiB LDS (attention)", 3072, 256, 18432, d, h);
  rc |= run_args(480, 512, d, h);
  rc |= run_args(256, 512, d, h);
  rc |= run_pre<1>(480, 512, d, h);
  rc |= run_pre<4>(480, 512, d, h);
  rc |= run_pre<8>(480, 512, d, h);
  rc |= run_pre<16>(480, 512, d, h);
  return rc;
}
