// Multi-head self-attention for short sequences (vision N = 50, text T = 77),
// gfx950.
//
// Replaces the attention subgraph of open_clip's ResidualAttentionBlock as
// exported by pull_onnx.py:53-68: softmax(Q K^T / sqrt(d) [+ causal mask]) V,
// per (sequence, head), head_dim d = 64.
//
// One 256-thread workgroup per (sequence, head).  K (row-major, XOR-swizzled)
// and V (transposed, padded rows) for the whole sequence sit in LDS; each wave
// owns 16-query tiles: S = Q K^T via 16x16x32 MFMA with the key on the lane,
// softmax in registers (row max / sum across the 16 lanes of a row group),
// unnormalised P -> LDS (16-bit), O = P V via MFMA, 1/rowsum applied in the
// epilogue.  Padded keys (>= N) and, for text, keys above the diagonal are
// masked to -inf (open_clip build_causal_mask: triu(-inf, 1)).
#include "common.hpp"
#include "kernels.hpp"

namespace clipgpu {

namespace {

template <typename T, int NKT>
__global__ __launch_bounds__(256) void attn_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                   int N, int H, int D, int causal) {
  typedef typename Vec8<T>::type V8;
  constexpr int NKP = NKT * 16;          // padded key count (multiple of 32)
  constexpr int ROW = NKP * 2 + 16;      // byte stride of Vt / P rows (odd # of 16B slots)
  constexpr int K_BYTES = NKP * 128;
  constexpr int VT_BYTES = 64 * ROW;
  constexpr int P_BYTES = 16 * ROW;
  __shared__ __attribute__((aligned(16))) char smem[K_BYTES + VT_BYTES + 4 * P_BYTES];
  char* const sK = smem;
  char* const sVt = smem + K_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const long ld = 3L * D;
  const T* base = qkv + (long)b * N * ld + h * 64;

  // K rows (swizzled) and V transposed into LDS; zero the padded keys.
  for (int q = tid; q < NKP * 8; q += 256) {
    const int r = q >> 3, c = q & 7;
    V8 kv, vv;
    if (r < N) {
      kv = *(const V8*)(base + (long)r * ld + D + c * 8);
      vv = *(const V8*)(base + (long)r * ld + 2 * D + c * 8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) { kv[e] = (T)0.f; vv[e] = (T)0.f; }
    }
    *(V8*)(sK + r * 128 + ((c ^ ((r >> 1) & 7)) << 4)) = kv;
#pragma unroll
    for (int e = 0; e < 8; ++e) *(T*)(sVt + (c * 8 + e) * ROW + r * 2) = vv[e];
  }
  __syncthreads();

  char* const sP = smem + K_BYTES + VT_BYTES + wave * P_BYTES;
  const int fr = lane & 15, fq = lane >> 4;
  const float scale = 0.125f;  // 1/sqrt(64)
  const int nqt = (N + 15) >> 4;

  for (int qt = wave; qt < nqt; qt += 4) {
    const int qrow_l = min(qt * 16 + fr, N - 1);
    V8 qa[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qa[kk] = *(const V8*)(base + (long)qrow_l * ld + kk * 32 + fq * 8);

    // S[q][key]: s[t][j] = S[qt*16 + fq*4 + j][t*16 + fr]
    f32x4 s[NKT];
#pragma unroll
    for (int t = 0; t < NKT; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int r = t * 16 + fr;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const V8 kb = *(const V8*)(sK + r * 128 + (((kk * 4 + fq) ^ (fr >> 1)) << 4));
        s[t] = mfma_16x16x32(qa[kk], kb, s[t]);
      }
    }

    float inv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int qrow = qt * 16 + fq * 4 + j;
      float m = -INFINITY;
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const int key = t * 16 + fr;
        float v = s[t][j] * scale;
        if (key >= N || (causal && key > qrow)) v = -INFINITY;
        s[t][j] = v;
        m = fmaxf(m, v);
      }
      m = group16_max(m);
      float sum = 0.f;
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const float e = __expf(s[t][j] - m);
        s[t][j] = e;
        sum += e;
      }
      sum = group16_sum(sum);
      inv[j] = 1.0f / sum;
    }

    // P (unnormalised) -> this wave's LDS rows.
#pragma unroll
    for (int t = 0; t < NKT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) *(T*)(sP + (fq * 4 + j) * ROW + (t * 16 + fr) * 2) = (T)s[t][j];
    __builtin_amdgcn_wave_barrier();

    // O = P V: o[ni][j] = O[qt*16 + fq*4 + j][ni*16 + fr]
    f32x4 o[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) o[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKP / 32; ++ks) {
      const V8 pa = *(const V8*)(sP + fr * ROW + (ks * 32 + fq * 8) * 2);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const V8 vb = *(const V8*)(sVt + (ni * 16 + fr) * ROW + (ks * 32 + fq * 8) * 2);
        o[ni] = mfma_16x16x32(pa, vb, o[ni]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = qt * 16 + fq * 4 + j;
      if (q >= N) continue;
      T* dst = out + ((long)b * N + q) * D + h * 64;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) dst[ni * 16 + fr] = (T)(o[ni][j] * inv[j]);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <typename T, int NKT>
hipError_t launch_nkt(const void* qkv, void* out, int B, int N, int H, int D, int causal, hipStream_t s) {
  hipLaunchKernelGGL((attn_kernel<T, NKT>), dim3(B * H), dim3(256), 0, s, (const T*)qkv, (T*)out, N, H,
                     D, causal);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_typed(const void* qkv, void* out, int B, int N, int H, int D, int causal, hipStream_t s) {
  const int nkt = ((N + 31) / 32) * 2;
  switch (nkt) {
    case 2: return launch_nkt<T, 2>(qkv, out, B, N, H, D, causal, s);
    case 4: return launch_nkt<T, 4>(qkv, out, B, N, H, D, causal, s);
    case 6: return launch_nkt<T, 6>(qkv, out, B, N, H, D, causal, s);
    case 8: return launch_nkt<T, 8>(qkv, out, B, N, H, D, causal, s);
    case 10: return launch_nkt<T, 10>(qkv, out, B, N, H, D, causal, s);
    case 12: return launch_nkt<T, 12>(qkv, out, B, N, H, D, causal, s);
    case 14: return launch_nkt<T, 14>(qkv, out, B, N, H, D, causal, s);
    case 16: return launch_nkt<T, 16>(qkv, out, B, N, H, D, causal, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_attention(DType dt, const void* qkv, void* out, int B, int N, int H, int D, int causal,
                            hipStream_t s) {
  if (N <= 0 || N > 256 || D != H * 64) return hipErrorInvalidValue;
  return dt == DT_BF16 ? launch_typed<__bf16>(qkv, out, B, N, H, D, causal, s)
                       : launch_typed<_Float16>(qkv, out, B, N, H, D, causal, s);
}

}  // namespace clipgpu
