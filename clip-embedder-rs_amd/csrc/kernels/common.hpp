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
typedef float f32x16 __attribute__((ext_vector_type(16)));
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

// Four consecutive residual-stream values (f32, or f16 when the stream is stored in f16:
// clipgpu_options.residual), widened to / rounded from f32.
__device__ __forceinline__ float4 ldx4(const float* p) { return *(const float4*)p; }
__device__ __forceinline__ float4 ldx4(const _Float16* p) {
  const f16x4 h = *(const f16x4*)p;
  return make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
}
__device__ __forceinline__ void stx4(float* p, float4 v) { *(float4*)p = v; }
__device__ __forceinline__ void stx4(_Float16* p, float4 v) {
  f16x4 h;
  h[0] = (_Float16)v.x; h[1] = (_Float16)v.y; h[2] = (_Float16)v.z; h[3] = (_Float16)v.w;
  *(f16x4*)p = h;
}

__device__ __forceinline__ f32x4 mfma_16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_16x16x32(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma_32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma_32x32x16(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) void lds_void;

// 16-byte global -> LDS DMA (global_load_lds_dwordx4).  The LDS destination is
// the wave-uniform `lds_base` + lane*16; the global source is per lane.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, (lds_void*)lds_base, 16, 0, 0);
}
// 4-byte form (global_load_lds_dword): lds_base + lane*4.
__device__ __forceinline__ void glds4(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, (lds_void*)lds_base, 4, 0, 0);
}

// ---- MX-fp8 (OCP e4m3fn elements, E8M0 scale per 32 consecutive elements of a row) ----
// Block exponent: the smallest e with amax <= 448 * 2^e (448 = largest e4m3 value, so no
// element saturates), from the bits of amax: amax = 1.f * 2^E, 448 = 1.75 * 2^8.  Clamped
// to the E8M0 range [-127, 127]; the stored scale byte is e + 127.
__device__ __forceinline__ int mx_exp(float amax) {
  const uint32_t b = __float_as_uint(amax);
  const int be = (int)(b >> 23);
  if (be == 0) return -127;  // zero / denormal block
  const int e = be - 135 + ((b & 0x7fffffu) > 0x600000u ? 1 : 0);
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}
// 2^-e (exact; 2^-127 is the f32 denormal 0x00400000)
__device__ __forceinline__ float mx_inv(int e) {
  return e < 127 ? __uint_as_float((uint32_t)(127 - e) << 23) : __uint_as_float(0x00400000u);
}
// four scaled values -> four e4m3 bytes (v_cvt_pk_fp8_f32: round to nearest even)
__device__ __forceinline__ uint32_t mx_pack4(float a, float b, float c, float d, float inv) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a * inv, b * inv, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c * inv, d * inv, w, true);
  return (uint32_t)w;
}

// Cross-lane reductions without the LDS permute unit (each __shfl_xor is a ds_bpermute
// round trip): inside a 16-lane row by DPP row rotations; between rows by the gfx950
// permlane swaps.  v_permlane16_swap(x, x) leaves rows {0,0,2,2} in the first result
// and {1,1,3,3} in the second, so (first op second) is x op x[lane ^ 16] in every lane;
// v_permlane32_swap likewise for lane ^ 32.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {  // sum over the 16 lanes of each row
  v += dpp_f32<0x128>(v);  // row_ror:8
  v += dpp_f32<0x124>(v);  // row_ror:4
  v += dpp_f32<0x122>(v);  // row_ror:2
  v += dpp_f32<0x121>(v);  // row_ror:1
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f32<0x128>(v));
  v = fmaxf(v, dpp_f32<0x124>(v));
  v = fmaxf(v, dpp_f32<0x122>(v));
  v = fmaxf(v, dpp_f32<0x121>(v));
  return v;
}
// v_permlane{16,32}_swap as inline asm: the swap writes both of its operands, and with the
// clang builtin this toolchain folded the second result into the first when the two were
// combined in one expression (x + x instead of x + x[lane ^ 16]; test_lane_reductions).
// The leading s_nop covers the VALU-write -> permlane-read hazard the compiler cannot see
// through the asm.
__device__ __forceinline__ void swap16(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void swap32(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ float xsum16(float v) {  // v + v[lane ^ 16]
  float a = v, b = v;
  swap16(a, b);
  return a + b;
}
__device__ __forceinline__ float xsum32(float v) {  // v + v[lane ^ 32]
  float a = v, b = v;
  swap32(a, b);
  return a + b;
}
__device__ __forceinline__ float xmax16(float v) {
  float a = v, b = v;
  swap16(a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float xmax32(float v) {
  float a = v, b = v;
  swap32(a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float wave_sum(float v) { return xsum32(xsum16(row16_sum(v))); }
__device__ __forceinline__ float wave_max(float v) { return xmax32(xmax16(row16_max(v))); }
// Reductions over the 16 lanes that share (lane >> 4): the row groups of a
// 16x16 MFMA accumulator (col = lane & 15).
__device__ __forceinline__ float group16_sum(float v) { return row16_sum(v); }
__device__ __forceinline__ float group16_max(float v) { return row16_max(v); }

// ---- LayerNorm fold (EPI_LNF, kernels/gemm.hip) ---------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));
// The folded LayerNorm + bias of one output from its row's (mean, rstd): rstd (acc - mean cs) + bias
__device__ __forceinline__ float lnf_out(float acc, float mean, float rstd, float cs, float bias) {
  return fmaf(fmaf(-mean, cs, acc), rstd, bias);
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
// x * sigmoid(z) given t = -z * log2(e) directly: one multiply less than fast_sigmoid_mul when the
// caller folds -log2(e) into its own constant (QuickGELU: t = x * (-1.702 * log2 e)).
__device__ __forceinline__ float sigmoid_mul_exp2(float x, float t) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(t));
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
#ifdef CLIPGPU_TEST_NO_ACT  // timing-experiment variant only (make variant): the activation skipped
  return x;
#endif
  if constexpr (ACT == ACT_QUICK_GELU) {
    return sigmoid_mul_exp2(x, x * -2.4554669596f);  // -1.702 * log2(e) (|rel err| 2^-24 of the product)
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
