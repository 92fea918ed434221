// Clip facade math for many images x many labels on the device:
//
//   logits[i][j] = dot(img[i], txt[j]).mul_add(logit_scale, logit_bias)      src/clip.rs:99-107
//   probs        = sigmoid(logits)                      (activation "sigmoid", :113-116)
//                | softmax over labels (axis 1)         (classify, :92-132)
//                | softmax over images (axis 0)         (rank_images, :134-170)
//   softmax: max-subtracted exp, divided by the sum      (:172-179)
//
// The dot products are exact-f32-input MFMA (v_mfma_f32_16x16x4_f32: f32 operands, f32
// accumulate; the 1/16-rate f32 matrix path, still ~10x the VALU FMA loop), 64 x 64 output
// tiles per 4-wave block, K staged through LDS 16 at a time.  The logit is one fmaf (Rust
// f32::mul_add); exp / divide are IEEE (expf, '/').  Embeddings are [n][E] row-major f32,
// E % 4 == 0.
#include "common.hpp"
#include "kernels.hpp"

namespace clipgpu {

namespace {

constexpr int TB = 64, TK = 16;

__device__ __forceinline__ float sigmoidf_ref(float l) { return 1.0f / (1.0f + expf(-l)); }

// Block: 64 images x 64 labels; wave w: rows (w >> 1) * 32, cols (w & 1) * 32 (2 x 2 MFMA tiles).
__global__ __launch_bounds__(256) void sim_logits_kernel(const float* __restrict__ img, const float* __restrict__ txt,
                                                         int ni, int nt, int E, float scale, float bias, int sigmoid,
                                                         float* __restrict__ out) {
  __shared__ float sA[TB][TK + 1];
  __shared__ float sB[TB][TK + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i0 = blockIdx.y * TB, j0 = blockIdx.x * TB;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // staging: thread -> (row tid / 4, k quad tid % 4)
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  const int ia = min(i0 + lr, ni - 1), jb = min(j0 + lr, nt - 1);
  for (int k0 = 0; k0 < E; k0 += TK) {
    const float4 va = *(const float4*)(img + (long)ia * E + k0 + lk);
    const float4 vb = *(const float4*)(txt + (long)jb * E + k0 + lk);
    __syncthreads();
    sA[lr][lk] = va.x; sA[lr][lk + 1] = va.y; sA[lr][lk + 2] = va.z; sA[lr][lk + 3] = va.w;
    sB[lr][lk] = vb.x; sB[lr][lk + 1] = vb.y; sB[lr][lk + 2] = vb.z; sB[lr][lk + 3] = vb.w;
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; kk += 4) {
      // 16x16x4: lane (r = lane & 15, q = lane >> 4) supplies A[r][q] and B[q][r]
      const int r = lane & 15, q = lane >> 4;
      float a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = sA[wr + t * 16 + r][kk + q];
        b[t] = sB[wc + t * 16 + r][kk + q];
      }
#pragma unroll
      for (int ta = 0; ta < 2; ++ta)
#pragma unroll
        for (int tb = 0; tb < 2; ++tb)
          acc[ta][tb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
    }
  }
  // C[row = 4 * (lane >> 4) + e][col = lane & 15]
#pragma unroll
  for (int ta = 0; ta < 2; ++ta)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = i0 + wr + ta * 16 + 4 * (lane >> 4) + e;
        const int j = j0 + wc + tb * 16 + (lane & 15);
        if (i < ni && j < nt) {
          const float l = fmaf(acc[ta][tb][e], scale, bias);
          out[(long)i * nt + j] = sigmoid ? sigmoidf_ref(l) : l;
        }
      }
}

// Softmax along rows (axis 1): one wave per row, any length.
__global__ __launch_bounds__(256) void softmax_rows_kernel(float* __restrict__ x, int rows, int n) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  float* p = x + (long)row * n;
  float m = -INFINITY;
  for (int j = lane; j < n; j += 64) m = fmaxf(m, p[j]);
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < n; j += 64) {
    const float e = expf(p[j] - m);
    p[j] = e;
    s += e;
  }
  s = wave_sum(s);
  for (int j = lane; j < n; j += 64) p[j] = p[j] / s;
}

// Softmax along columns (axis 0): one thread per column, rows walked in order (coalesced
// across the threads of a block).
__global__ __launch_bounds__(256) void softmax_cols_kernel(float* __restrict__ x, int rows, int n) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  float m = -INFINITY;
  for (int i = 0; i < rows; ++i) m = fmaxf(m, x[(long)i * n + j]);
  float s = 0.f;
  for (int i = 0; i < rows; ++i) {
    const float e = expf(x[(long)i * n + j] - m);
    x[(long)i * n + j] = e;
    s += e;
  }
  for (int i = 0; i < rows; ++i) x[(long)i * n + j] = x[(long)i * n + j] / s;
}

}  // namespace

hipError_t launch_similarity(const float* img, int ni, const float* txt, int nt, int E, float scale, float bias,
                             int activation, int axis, float* out, hipStream_t s) {
  if (ni <= 0 || nt <= 0 || E <= 0 || E % TK != 0 || ni > 65535 * TB) return hipErrorInvalidValue;
  if (activation < SIM_SOFTMAX || activation > SIM_LOGITS || axis < 0 || axis > 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sim_logits_kernel, dim3((nt + TB - 1) / TB, (ni + TB - 1) / TB), dim3(256), 0, s, img, txt, ni, nt,
                     E, scale, bias, activation == SIM_SIGMOID ? 1 : 0, out);
  if (activation == SIM_SOFTMAX) {
    if (axis == 1)
      hipLaunchKernelGGL(softmax_rows_kernel, dim3((ni + 3) / 4), dim3(256), 0, s, out, ni, nt);
    else
      hipLaunchKernelGGL(softmax_cols_kernel, dim3((nt + 255) / 256), dim3(256), 0, s, out, ni, nt);
  }
  return hipGetLastError();
}

}  // namespace clipgpu
