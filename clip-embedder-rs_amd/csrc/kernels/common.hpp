// Shared device-side types and helpers for the clipgpu gfx950 kernels.
//
// Data layout conventions (see DESIGN.md §Data layout):
//   * residual stream  x : f32   [rows][D]      rows = B * tokens, row-major
//   * GEMM operands    A : T16   [rows][K]      K-contiguous
//                      W : T16   [N][K]         (torch Linear layout, "B^T")
//   * T16 is __bf16 (default) or _Float16, selected per engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace clipgpu {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

template <typename T> struct Vec8;
template <> struct Vec8<__bf16> { typedef bf16x8 type; };
template <> struct Vec8<_Float16> { typedef f16x8 type; };
template <typename T> struct Vec4;
template <> struct Vec4<__bf16> { typedef bf16x4 type; };
template <> struct Vec4<_Float16> { typedef f16x4 type; };

__device__ __forceinline__ f32x4 mfma_16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_16x16x32(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) void lds_void;

// 16-byte global -> LDS DMA (global_load_lds_dwordx4).  The LDS destination is
// the wave-uniform `lds_base` + lane*16; the global source is per lane.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, (lds_void*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Reductions over the 16 lanes that share (lane >> 4): the row groups of a
// 16x16 MFMA accumulator (col = lane & 15).
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Activations (epilogue of c_fc).  Reference semantics: open_clip QuickGELU
// x*sigmoid(1.702x) for OpenAI-style configs, nn.GELU (erf) otherwise,
// tanh-GELU for SigLIP.
enum Act { ACT_NONE = 0, ACT_QUICK_GELU = 1, ACT_GELU = 2, ACT_GELU_TANH = 3 };

// Epilogue-cost forms (the GEMM epilogue evaluates one per output element; the 16-bit
// output rounding, 2^-9 relative, dwarfs their error):
//   QuickGELU  x * sigmoid(1.702 x)                 v_exp + v_rcp
//   tanh-GELU  0.5 x (1 + tanh(u)) == x * sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3):
//              the same v_exp + v_rcp (exact identity; tanhf is a long library call)
//   erf-GELU   0.5 x (1 + erf(x / sqrt 2)), erf by Abramowitz-Stegun 7.1.26 (|err| <= 1.5e-7:
//              one v_rcp, one v_exp, five FMAs) instead of the library erff
__device__ __forceinline__ float fast_sigmoid_mul(float x, float z) {  // x * sigmoid(z)
  return x * __builtin_amdgcn_rcpf(1.0f + __expf(-z));
}
__device__ __forceinline__ float fast_erf(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = 1.0f - p * t * __expf(-ax * ax);
  return copysignf(y, x);
}

template <int ACT>
__device__ __forceinline__ float apply_act(float x) {
  if constexpr (ACT == ACT_QUICK_GELU) {
    return fast_sigmoid_mul(x, 1.702f * x);
  } else if constexpr (ACT == ACT_GELU) {
    return 0.5f * x * (1.0f + fast_erf(x * 0.70710678118654752f));
  } else if constexpr (ACT == ACT_GELU_TANH) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    return fast_sigmoid_mul(x, 2.0f * k0 * fmaf(k1 * x, x * x, x));
  } else {
    return x;
  }
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks b, b+8, b+16 ... (which the dispatcher places on
// one XCD) receive a contiguous range of tile ids, so tiles sharing operand
// panels share that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int pid, int nwg) {
  const int xcd = pid & 7, q = nwg >> 3, r = nwg & 7;
  const int start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + (pid >> 3);
}

}  // namespace clipgpu
