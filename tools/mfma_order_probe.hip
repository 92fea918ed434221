// Probe: does a chain of v_mfma_f32_32x32x16_bf16 give the same f32 bits as a chain of
// v_mfma_f32_16x16x32_bf16 over the same K order?  (If it does, the trunk GEMMs could switch to
// the 32x32 MFMA -- which holds the SIMD's vector issue for 8 of 32 cycles instead of 8 of 16 --
// without changing any output bit.)  Standalone: hipcc --offload-arch=gfx950 -O3 -o probe
// tools/mfma_order_probe.hip && ./probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// A [32][K], B [32][K] (both K-contiguous), C[i][j] = sum_k A[i][k] B[j][k]
template <typename T> struct V8T;
template <> struct V8T<__bf16> { typedef bf16x8 t; };
template <> struct V8T<_Float16> { typedef f16x8 t; };
__device__ inline f32x4 m16(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
__device__ inline f32x4 m16(f16x8 a, f16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
__device__ inline f32x16 m32(bf16x8 a, bf16x8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }
__device__ inline f32x16 m32(f16x8 a, f16x8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0); }

template <typename T>
__global__ void mfma16(const T* A, const T* B, float* C, int K) {
  typedef typename V8T<T>::t V8;
  const int lane = threadIdx.x;
  const int fr = lane & 15, fq = lane >> 4;
  for (int bi = 0; bi < 2; ++bi)
    for (int bj = 0; bj < 2; ++bj) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k0 = 0; k0 < K; k0 += 32) {
        V8 a, b;
        for (int e = 0; e < 8; ++e) {
          a[e] = A[(bi * 16 + fr) * K + k0 + fq * 8 + e];
          b[e] = B[(bj * 16 + fr) * K + k0 + fq * 8 + e];
        }
        // operand roles as the product kernels: W (B rows) is the MFMA "A" operand
        acc = m16(b, a, acc);
      }
      // acc[j] = C[row = bi*16 + fr][col = bj*16 + fq*4 + j]
      for (int j = 0; j < 4; ++j) C[(bi * 16 + fr) * 32 + bj * 16 + fq * 4 + j] = acc[j];
    }
}

template <typename T>
__global__ void mfma32(const T* A, const T* B, float* C, int K, int korder) {
  typedef typename V8T<T>::t V8;
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc;
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  for (int k0 = 0; k0 < K; k0 += 16) {
    V8 a, b;
    for (int e = 0; e < 8; ++e) {
      // korder 0: lane half h takes k0 + 8h + e; 1: the 16x16x32 pairing (k0/32 block, halves interleaved)
      const int k = korder == 0 ? k0 + h * 8 + e : k0 + h * 8 + e;
      a[e] = A[r * K + k];
      b[e] = B[r * K + k];
    }
    acc = m32(b, a, acc);
  }
  // D (32x32): lane (r, h), register j -> row-of-A-operand... written back both ways by the host check
  for (int j = 0; j < 16; ++j) {
    const int dr = 8 * (j / 4) + 4 * h + (j % 4);  // the "A" (= B-matrix) operand row index
    C[r * 32 + dr] = acc[j];                      // C[A row r][B row dr]
  }
}

template <typename T>
void run(int K, unsigned seed, long& same, long& total, double& maxrel) {
  std::mt19937 g(seed);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<T> A(32 * K), B(32 * K);
  for (auto& x : A) x = (T)(nd(g) * (seed % 3 == 0 ? 100.f : 1.f));
  for (auto& x : B) x = (T)(nd(g) / std::sqrt((float)K));
  T *dA, *dB;
  float *d16, *d32;
  (void)hipMalloc(&dA, A.size() * sizeof(T));
  (void)hipMalloc(&dB, B.size() * sizeof(T));
  (void)hipMalloc(&d16, 32 * 32 * 4);
  (void)hipMalloc(&d32, 32 * 32 * 4);
  (void)hipMemcpy(dA, A.data(), A.size() * sizeof(T), hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), B.size() * sizeof(T), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mfma16<T>, dim3(1), dim3(64), 0, 0, dA, dB, d16, K);
  hipLaunchKernelGGL(mfma32<T>, dim3(1), dim3(64), 0, 0, dA, dB, d32, K, 0);
  std::vector<float> c16(1024), c32(1024);
  (void)hipMemcpy(c16.data(), d16, 4096, hipMemcpyDeviceToHost);
  (void)hipMemcpy(c32.data(), d32, 4096, hipMemcpyDeviceToHost);
  for (int i = 0; i < 1024; ++i) {
    const float a = c16[i], b = c32[i];
    same += std::memcmp(&a, &b, 4) == 0;
    ++total;
    maxrel = std::fmax(maxrel, std::fabs((double)a - b) / (std::fabs((double)a) + 1e-12));
  }
  (void)hipFree(dA); (void)hipFree(dB); (void)hipFree(d16); (void)hipFree(d32);
}

int main() {
  for (int dt = 0; dt < 2; ++dt)
    for (int K : {32, 128, 768, 3072, 5120}) {
      long same = 0, total = 0;
      double maxrel = 0;
      for (unsigned seed = 1; seed <= 12; ++seed) {
        if (dt == 0) run<__bf16>(K, seed, same, total, maxrel);
        else run<_Float16>(K, seed, same, total, maxrel);
      }
      std::printf("%s K=%5d: mfma 16x16x32 vs 32x32x16 chains: %ld / %ld outputs bit-identical, max rel diff %.3e\n",
                  dt == 0 ? "bf16" : "f16 ", K, same, total, maxrel);
    }
  return 0;
}
