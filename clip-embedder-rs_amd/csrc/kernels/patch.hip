// Patch rows: the GEMM A operand of the patch-embedding conv (a9), written by one
// streaming pass over the pixels.
//
//   rows[b*G*G + py*G + px][k] = pixel(b, ch, py*P + ky, px*P + kx),   k = ch*P*P + ky*P + kx
//   (k >= 3*P*P: 0, the zero-padded K of the 16-bit conv weight)
//
// conv1 (kernel = stride = P, no padding) is exactly this row layout times the
// weight [D][3*P*P]^T.  The source is either the normalised f32 NCHW batch of
// preprocess_batch (src/vision.rs:119-140) or u8 NHWC pixels normalised on the
// fly exactly as normalize_pixels (src/vision.rs:235-259: (p / 255 - mean[c]) /
// std[c] in f32, divide not reciprocal-multiply) -- so both inputs give the same
// 16-bit rows, bit for bit.
//
// Why a pass and not a gather inside the GEMM: the pixels are read once from HBM
// here, by enough waves to cover HBM latency, and the GEMM then streams 16-bit
// rows through its LDS-DMA pipeline like every other trunk GEMM.  The earlier
// in-GEMM gather (register-staged, one K-step of latency cover, ~1 block per CU
// at M = 128 x 49) ran at 92 TFLOP/s: 13 % of the ViT-B/32 step.
//
// One thread writes one 16-byte chunk (8 consecutive k of one row): with P % 8 == 0
// those are 8 pixels of one image row (f32: two float4 loads; u8 NHWC: three
// 8-byte loads of the 8 RGB triples, every channel's byte picked out).
#include "common.hpp"
#include "kernels.hpp"

namespace clipgpu {

namespace {

template <typename T, int SRC>
__global__ __launch_bounds__(256) void patch_rows_kernel(const void* __restrict__ img, float m0, float m1, float m2,
                                                         float s0, float s1, float s2, T* __restrict__ out, long nchunks,
                                                         int S, int P, int G, int Kv, int Kp) {
  typedef typename Vec8<T>::type V8;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nchunks) return;
  const int cpr = Kp >> 3;
  const long m = t / cpr;
  const int k0 = (int)(t - m * cpr) * 8;
  const int G2 = G * G;
  const long b = m / G2;
  const int pp = (int)(m - b * G2), py = pp / G, px = pp - py * G;
  const int PP = P * P;
  float v[8];
  auto mean_of = [&](int ch) { return ch == 0 ? m0 : (ch == 1 ? m1 : m2); };
  auto std_of = [&](int ch) { return ch == 0 ? s0 : (ch == 1 ? s1 : s2); };
  if ((P & 7) == 0 && k0 + 8 <= Kv) {
    const int ch = k0 / PP, rem = k0 - ch * PP, ky = rem / P, kx = rem - ky * P;
    const long y = (long)py * P + ky, x = (long)px * P + kx;
    if constexpr (SRC == A_IMG_F32) {
      const float* src = (const float*)img + ((b * 3 + ch) * S + y) * S + x;
      const float4 a = *(const float4*)src, c = *(const float4*)(src + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
      v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
    } else {
      const uint8_t* src = (const uint8_t*)img + ((b * S + y) * S + x) * 3;  // 24 B, 8-byte aligned
      uint8_t px8[24];
      const uint64_t* s64 = (const uint64_t*)src;
#pragma unroll
      for (int i = 0; i < 3; ++i) *(uint64_t*)(px8 + 8 * i) = s64[i];
      const float mu = mean_of(ch), sd = std_of(ch);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ((float)px8[e * 3 + ch] / 255.0f - mu) / sd;
    }
  } else {  // P % 8 != 0 (patch 14) or the K tail / zero padding
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = k0 + e;
      float val = 0.f;
      if (k < Kv) {
        const int ch = k / PP, rem = k - ch * PP, ky = rem / P, kx = rem - ky * P;
        const long y = (long)py * P + ky, x = (long)px * P + kx;
        if constexpr (SRC == A_IMG_F32) {
          val = ((const float*)img)[((b * 3 + ch) * S + y) * S + x];
        } else {
          const float u = (float)((const uint8_t*)img)[((b * S + y) * S + x) * 3 + ch] / 255.0f;
          val = (u - mean_of(ch)) / std_of(ch);
        }
      }
      v[e] = val;
    }
  }
  V8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (T)v[e];
  *(V8*)(out + m * Kp + k0) = o;
}

template <typename T>
hipError_t launch_typed(int src, const void* img, const float* mean, const float* stdv, void* out, int B, int S,
                        int P, int Kv, int Kp, hipStream_t s) {
  const int G = S / P;
  const long nchunks = (long)B * G * G * (Kp / 8);
  const int blocks = (int)((nchunks + 255) / 256);
  const float m0 = mean ? mean[0] : 0.f, m1 = mean ? mean[1] : 0.f, m2 = mean ? mean[2] : 0.f;
  const float s0 = stdv ? stdv[0] : 1.f, s1 = stdv ? stdv[1] : 1.f, s2 = stdv ? stdv[2] : 1.f;
  if (src == A_IMG_F32)
    hipLaunchKernelGGL((patch_rows_kernel<T, A_IMG_F32>), dim3(blocks), dim3(256), 0, s, img, m0, m1, m2, s0, s1, s2,
                       (T*)out, nchunks, S, P, G, Kv, Kp);
  else
    hipLaunchKernelGGL((patch_rows_kernel<T, A_IMG_U8>), dim3(blocks), dim3(256), 0, s, img, m0, m1, m2, s0, s1, s2,
                       (T*)out, nchunks, S, P, G, Kv, Kp);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_patch_rows(DType dt, int src, const void* img, const float* mean, const float* stdv, void* out,
                             int B, int S, int P, int Kv, int Kp, hipStream_t s) {
  if (B <= 0 || P <= 0 || S % P != 0 || Kp % 64 != 0 || Kv > Kp || Kv != 3 * P * P) return hipErrorInvalidValue;
  if (src != A_IMG_F32 && src != A_IMG_U8) return hipErrorInvalidValue;
  return dt == DT_BF16 ? launch_typed<__bf16>(src, img, mean, stdv, out, B, S, P, Kv, Kp, s)
                       : launch_typed<_Float16>(src, img, mean, stdv, out, B, S, P, Kv, Kp, s);
}

}  // namespace clipgpu
