// Multi-head self-attention, gfx950: a whole-sequence-in-LDS kernel for short
// sequences (vision N = 50, text T = 77; head dim 64) and a tiled online-softmax
// kernel for long ones / head dims 72, 80 (flash_attn_kernel below).
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


// ---------------------------------------------------------------------------
// Tiled ("flash") attention for long sequences and head dims 64 / 72 / 80:
// SigLIP2-384 (576 tokens, d 72), ViT-H/14-378 (730 tokens, d 80).
//
// One 256-thread workgroup per (sequence, head, 64-query block); each wave owns
// 16 queries.  Keys/values stream through LDS in tiles of 64 (K row-major, V
// transposed; row strides of an odd number of 16-byte slots), S = Q K^T by
// 16x16x32 MFMA with the head dim zero-padded to HK = 64 / 96, online softmax
// (running row max m and sum l; O and l rescaled by exp(m_old - m_new)), P to
// LDS, O += P V with the head dim padded to HV = 64 / 80.  Causal: tiles past
// the block's last query are skipped, keys > query masked.
// ---------------------------------------------------------------------------
template <typename T, int HD>
__global__ __launch_bounds__(256) void flash_attn_kernel(const T* __restrict__ qkv, T* __restrict__ out, int N,
                                                         int H, int D, int causal, float scale) {
  typedef typename Vec8<T>::type V8;
  constexpr int HK = (HD + 31) / 32 * 32, HV = (HD + 15) / 16 * 16;
  constexpr int KT = 64;                      // keys per tile
  constexpr int KROW = HK * 2 + 16;           // bytes: K rows
  constexpr int VROW = KT * 2 + 16;           // bytes: V^T and P rows
  constexpr int CH = HD / 8;                  // 16-byte chunks per head row
  __shared__ __attribute__((aligned(16))) char smem[KT * KROW + HV * VROW + 4 * 16 * VROW];
  char* const sK = smem;
  char* const sVt = smem + KT * KROW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nqb = (N + 63) / 64;
  const int qb = blockIdx.x % nqb, bh = blockIdx.x / nqb;
  const int b = bh / H, h = bh % H;
  const long ld = 3L * D;
  const T* base = qkv + (long)b * N * ld + (long)h * HD;
  char* const sP = smem + KT * KROW + HV * VROW + wave * 16 * VROW;
  const int fr = lane & 15, fq = lane >> 4;

  // zero the padding that tile loads never write: K head-dim pad, V^T pad rows
  if constexpr (HK > HD) {
    constexpr int PADC = HK / 8 - CH;
    for (int q = tid; q < KT * PADC; q += 256) *(V8*)(sK + (q / PADC) * KROW + (CH + q % PADC) * 16) = V8{};
  }
  if constexpr (HV > HD)
    for (int q = tid; q < (HV - HD) * KT; q += 256) *(T*)(sVt + (HD + q / KT) * VROW + (q % KT) * 2) = (T)0.f;

  // this wave's 16 queries: Q fragments (head dim zero-padded to HK)
  const int q0 = qb * 64 + wave * 16;
  V8 qa[HK / 32];
  {
    const int qr = min(q0 + fr, N - 1);
#pragma unroll
    for (int kk = 0; kk < HK / 32; ++kk) {
      const int c = kk * 4 + fq;
      qa[kk] = c < CH ? *(const V8*)(base + (long)qr * ld + c * 8) : V8{};
    }
  }
  f32x4 o[HV / 16];
#pragma unroll
  for (int ni = 0; ni < HV / 16; ++ni) o[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[j] = -INFINITY;
    l[j] = 0.f;
  }

  const int last_key = causal ? min(N, qb * 64 + 64) : N;
  const int ntiles = (last_key + KT - 1) / KT;
  for (int kt = 0; kt < ntiles; ++kt) {
    __syncthreads();  // previous tile fully consumed
    for (int q = tid; q < KT * CH; q += 256) {
      const int r = q / CH, c = q % CH, key = kt * KT + r;
      V8 kv{}, vv{};
      if (key < N) {
        kv = *(const V8*)(base + (long)key * ld + D + c * 8);
        vv = *(const V8*)(base + (long)key * ld + 2 * D + c * 8);
      }
      *(V8*)(sK + r * KROW + c * 16) = kv;
#pragma unroll
      for (int e = 0; e < 8; ++e) *(T*)(sVt + (c * 8 + e) * VROW + r * 2) = vv[e];
    }
    __syncthreads();

    // S[q][key]: s[t][j] = S[q0 + fq*4 + j][kt*64 + t*16 + fr]
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < HK / 32; ++kk) {
        const V8 kb = *(const V8*)(sK + (t * 16 + fr) * KROW + (kk * 4 + fq) * 16);
        s[t] = mfma_16x16x32(qa[kk], kb, s[t]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int qrow = q0 + fq * 4 + j;
      float mt = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int key = kt * KT + t * 16 + fr;
        float v = s[t][j] * scale;
        if (key >= N || (causal && key > qrow)) v = -INFINITY;
        s[t][j] = v;
        mt = fmaxf(mt, v);
      }
      mt = group16_max(mt);
      const float mn = fmaxf(m[j], mt);
      const float corr = __expf(m[j] - mn);  // m[j] = -inf on the first tile: 0
      float sum = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float e = __expf(s[t][j] - mn);
        s[t][j] = e;
        sum += e;
      }
      l[j] = l[j] * corr + group16_sum(sum);
      m[j] = mn;
#pragma unroll
      for (int ni = 0; ni < HV / 16; ++ni) o[ni][j] *= corr;
    }
    // P -> this wave's LDS rows, then O += P V
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) *(T*)(sP + (fq * 4 + j) * VROW + (t * 16 + fr) * 2) = (T)s[t][j];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int ks = 0; ks < KT / 32; ++ks) {
      const V8 pa = *(const V8*)(sP + fr * VROW + (ks * 32 + fq * 8) * 2);
#pragma unroll
      for (int ni = 0; ni < HV / 16; ++ni) {
        const V8 vb = *(const V8*)(sVt + (ni * 16 + fr) * VROW + (ks * 32 + fq * 8) * 2);
        o[ni] = mfma_16x16x32(pa, vb, o[ni]);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = q0 + fq * 4 + j;
    if (q >= N) continue;
    const float inv = 1.0f / l[j];
    T* dst = out + ((long)b * N + q) * D + (long)h * HD;
#pragma unroll
    for (int ni = 0; ni < HV / 16; ++ni) {
      const int d = ni * 16 + fr;
      if (d < HD) dst[d] = (T)(o[ni][j] * inv);
    }
  }
}

template <typename T, int HD>
hipError_t launch_flash(const void* qkv, void* out, int B, int N, int H, int D, int causal, hipStream_t s) {
  const int nqb = (N + 63) / 64;
  hipLaunchKernelGGL((flash_attn_kernel<T, HD>), dim3(B * H * nqb), dim3(256), 0, s, (const T*)qkv, (T*)out, N, H, D,
                     causal, 1.0f / sqrtf((float)HD));
  return hipGetLastError();
}

template <typename T>
hipError_t launch_flash_hd(const void* qkv, void* out, int B, int N, int H, int D, int causal, hipStream_t s) {
  switch (D / H) {
    case 64: return launch_flash<T, 64>(qkv, out, B, N, H, D, causal, s);
    case 72: return launch_flash<T, 72>(qkv, out, B, N, H, D, causal, s);
    case 80: return launch_flash<T, 80>(qkv, out, B, N, H, D, causal, s);
  }
  return hipErrorInvalidValue;
}

// MAP attention pool (timm AttentionPoolLatent; oracle/clip_ref.py encode_image_siglip): one
// learned query per head over the N tokens of one image.  One 256-thread block per (image,
// head): scores by threads over keys, block softmax, then waves split the keys and lanes
// the head dims for o = sum_n p_n v_n.  Memory-bound and tiny next to the trunk.
template <typename T>
__global__ __launch_bounds__(256) void map_attn_kernel(const float* __restrict__ q, const T* __restrict__ kv,
                                                       T* __restrict__ out, int N, int H, int D, float scale) {
  __shared__ float sS[1024];
  __shared__ float sO[4][128];
  __shared__ float red[4];
  const int b = blockIdx.x / H, h = blockIdx.x % H, hd = D / H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* kvb = kv + (long)b * N * 2 * D;
  const float* qh = q + (long)h * hd;
  float lmax = -INFINITY;
  for (int n = tid; n < N; n += 256) {
    const T* kr = kvb + (long)n * 2 * D + (long)h * hd;
    float s = 0.f;
    for (int d = 0; d < hd; ++d) s += qh[d] * (float)kr[d];
    s *= scale;
    sS[n] = s;
    lmax = fmaxf(lmax, s);
  }
  lmax = wave_max(lmax);
  if (lane == 0) red[wave] = lmax;
  __syncthreads();
  const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float lsum = 0.f;
  for (int n = tid; n < N; n += 256) {
    const float e = __expf(sS[n] - m);
    sS[n] = e;
    lsum += e;
  }
  lsum = wave_sum(lsum);
  if (lane == 0) red[wave] = lsum;
  __syncthreads();
  const float inv = 1.0f / (red[0] + red[1] + red[2] + red[3]);
  float o0 = 0.f, o1 = 0.f;
  for (int n = wave; n < N; n += 4) {
    const T* vr = kvb + (long)n * 2 * D + D + (long)h * hd;
    const float pn = sS[n];
    if (lane < hd) o0 += pn * (float)vr[lane];
    if (lane + 64 < hd) o1 += pn * (float)vr[lane + 64];
  }
  sO[wave][lane] = o0;
  sO[wave][lane + 64] = o1;
  __syncthreads();
  if (tid < hd) out[(long)b * D + (long)h * hd + tid] = (T)((sO[0][tid] + sO[1][tid] + sO[2][tid] + sO[3][tid]) * inv);
}

}  // namespace

hipError_t launch_map_attention(DType dt, const float* q, const void* kv, void* out, int B, int N, int H, int D,
                                hipStream_t s) {
  if (B <= 0 || N <= 0 || N > 1024 || H <= 0 || D % H || D / H > 128) return hipErrorInvalidValue;
  const float scale = 1.0f / sqrtf((float)(D / H));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(map_attn_kernel<__bf16>, dim3(B * H), dim3(256), 0, s, q, (const __bf16*)kv, (__bf16*)out, N, H,
                       D, scale);
  else
    hipLaunchKernelGGL(map_attn_kernel<_Float16>, dim3(B * H), dim3(256), 0, s, q, (const _Float16*)kv,
                       (_Float16*)out, N, H, D, scale);
  return hipGetLastError();
}

hipError_t launch_attention(DType dt, const void* qkv, void* out, int B, int N, int H, int D, int causal,
                            hipStream_t s) {
  if (N <= 0 || H <= 0 || D % H) return hipErrorInvalidValue;
  if (D == H * 64 && N <= 256)  // whole sequence in LDS (ViT-B/32 vision N = 50, CLIP text T = 77)
    return dt == DT_BF16 ? launch_typed<__bf16>(qkv, out, B, N, H, D, causal, s)
                         : launch_typed<_Float16>(qkv, out, B, N, H, D, causal, s);
  return dt == DT_BF16 ? launch_flash_hd<__bf16>(qkv, out, B, N, H, D, causal, s)
                       : launch_flash_hd<_Float16>(qkv, out, B, N, H, D, causal, s);
}

}  // namespace clipgpu
