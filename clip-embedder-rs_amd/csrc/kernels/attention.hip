// Multi-head self-attention, gfx950: a whole-sequence-in-LDS kernel for short
// sequences (vision N = 50, text T = 77; head dim 64) and a tiled online-softmax
// kernel for long ones / head dims 72, 80 (flash_attn_kernel below).
//
// Replaces the attention subgraph of open_clip's ResidualAttentionBlock as
// exported by pull_onnx.py:53-68: softmax(Q K^T / sqrt(d) [+ causal mask]) V,
// per (sequence, head), head_dim d = 64.
//
// One workgroup per (sequence, head), one wave per 16-query tile (up to 8; more
// tiles are walked by 4 waves), so N = 77 runs 5 waves instead of 4 waves with one
// taking two tiles.  K (row-major, XOR-swizzled) and V (row-major, 160-byte rows) for
// the whole sequence sit in LDS; each wave computes the transposed products of flash_attn_kernel
// below: S^T = K Q^T (16x16x32 MFMA; lane (fr, fq) holds query fr's scores for
// keys t*16 + 4fq + j, so the row max / sum are in-lane plus two xor-shuffles),
// O^T = V^T P^T with V^T read by ds_read_b64_tr_b16 and P^T taken straight from
// the S^T accumulators (a key order both operands share), 1/rowsum in the
// epilogue, 8-byte stores of 4 head dims.  Padded keys (>= N) and, for text,
// keys above the diagonal are masked to -inf (open_clip build_causal_mask:
// triu(-inf, 1)); causal key tiles wholly above the query tile's diagonal are skipped
// (their probabilities are exactly 0).
#include <type_traits>

#include "common.hpp"
#include "kernels.hpp"

namespace clipgpu {

namespace {

// ds_read_b64_tr_b16 (16-bit lanes; the i16 form, reinterpreted as T): per 16-lane group,
// lane 4q+p addresses row q, columns 4p..4p+3 of a 4 x 16 block; lane i receives column i.
template <typename T>
struct TrRead {
  typedef T V4 __attribute__((ext_vector_type(4)));
  typedef short I4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ V4 read(const char* p) {
    return __builtin_bit_cast(V4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) I4*)p));
  }
};

template <typename T, int NKT>
__global__ __launch_bounds__(512) void attn_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                   int N, int H, int D, int causal) {
  typedef typename Vec8<T>::type V8;
  typedef typename Vec4<T>::type V4;
  typedef typename TrRead<T>::V4 TR4;
  constexpr int NKP = NKT * 16;          // padded key count (multiple of 32)
  constexpr int VROW = 160;              // V rows: 40 banks (conflict-free transposed reads)
  constexpr int K_BYTES = NKP * 128;
  __shared__ __attribute__((aligned(16))) char smem[K_BYTES + NKP * VROW];
  char* const sK = smem;
  char* const sV = smem + K_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = blockDim.x >> 6;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const long ld = 3L * D;
  const T* base = qkv + (long)b * N * ld + h * 64;

  // K rows (swizzled) and V rows into LDS; zero the padded keys.
  for (int q = tid; q < NKP * 8; q += blockDim.x) {
    const int r = q >> 3, c = q & 7;
    V8 kv{}, vv{};
    if (r < N) {
      kv = *(const V8*)(base + (long)r * ld + D + c * 8);
      vv = *(const V8*)(base + (long)r * ld + 2 * D + c * 8);
    }
    *(V8*)(sK + r * 128 + ((c ^ ((r >> 1) & 7)) << 4)) = kv;
    *(V8*)(sV + r * VROW + c * 16) = vv;
  }
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  const float scale_log2 = 0.125f * 1.4426950408889634f;  // 1/sqrt(64), base-2 softmax
  const int nqt = (N + 15) >> 4;

  for (int qt = wave; qt < nqt; qt += nwaves) {
    // causal: keys past this tile's last query (qt*16 + 15) have probability 0
    const int kt_end = causal ? qt + 1 : NKT;
    const int q = qt * 16 + fr;
    const int qrow_l = min(q, N - 1);
    V8 qf[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qf[kk] = *(const V8*)(base + (long)qrow_l * ld + kk * 32 + fq * 8);

    // S^T: s[t][j] = S[query q][key t*16 + 4fq + j]
    f32x4 s[NKT];
#pragma unroll
    for (int t = 0; t < NKT; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t >= kt_end) continue;  // (masked to -inf below)
      const int r = t * 16 + fr;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const V8 ka = *(const V8*)(sK + r * 128 + (((kk * 4 + fq) ^ (fr >> 1)) << 4));
        s[t] = mfma_16x16x32(ka, qf[kk], s[t]);
      }
    }
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < NKT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = t * 16 + 4 * fq + j;
        float v = s[t][j] * scale_log2;
        if (key >= N || (causal && key > q)) v = -INFINITY;
        s[t][j] = v;
        m = fmaxf(m, v);
      }
    m = xmax32(xmax16(m));
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < NKT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float e = exp2f(s[t][j] - m);
        s[t][j] = e;
        sum += e;
      }
    sum = xsum32(xsum16(sum));

    // O^T[d][q] = V^T P^T; k order of step ks: element e of quarter fq <-> key 32ks + 16(e>>2) + 4fq + (e&3)
    f32x4 o[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) o[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKP / 32; ++ks) {
      if (2 * ks >= kt_end) continue;  // all 32 keys of the step have P = 0
      V8 pf;
#pragma unroll
      for (int e = 0; e < 8; ++e) pf[e] = (T)s[2 * ks + (e >> 2)][e & 3];
      const char* const va0 = sV + (32 * ks + 4 * fq + (fr >> 2)) * VROW + 8 * (fr & 3);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const TR4 lo = TrRead<T>::read(va0 + ni * 32);
        const TR4 hi = TrRead<T>::read(va0 + 16 * VROW + ni * 32);
        V8 va;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          va[e] = lo[e];
          va[e + 4] = hi[e];
        }
        o[ni] = mfma_16x16x32(va, pf, o[ni]);
      }
    }
    if (q < N) {
      const float inv = 1.0f / sum;
      T* dst = out + ((long)b * N + q) * D + h * 64;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        V4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (T)(o[ni][j] * inv);
        *(V4*)(dst + ni * 16 + 4 * fq) = w;
      }
    }
  }
}

template <typename T, int NKT>
hipError_t launch_nkt(const void* qkv, void* out, int B, int N, int H, int D, int causal, hipStream_t s) {
  const int nqt = (N + 15) / 16;
  const int waves = nqt <= 8 ? nqt : 4;
  hipLaunchKernelGGL((attn_kernel<T, NKT>), dim3(B * H), dim3(64 * waves), 0, s, (const T*)qkv, (T*)out, N, H,
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
// One 256-thread workgroup per (sequence, head, 128-query block); each wave owns
// 32 queries as two 16-query MFMA blocks.  Keys/values stream through LDS in
// tiles of 64, double-buffered: tile kt+1 is loaded into registers while tile kt
// is computed and written to the other buffer behind one barrier per tile.
//
// Transposed products, so nothing but K and V ever touches LDS:
//   S^T = K Q^T   (16x16x32 MFMA, A = K rows, B = Q; head dim zero-padded to HK)
//     -> lane (fr, fq) holds the scores of query fr for keys t*16 + 4fq + j:
//        the online-softmax row statistics of query fr live in that lane
//        (max / sum across the 4 lanes of a column: two xor-shuffles);
//   O^T += V^T P^T (A = V^T by ds_read_b64_tr_b16 from the row-major V tile,
//        B = P^T straight from the S^T accumulators in a permuted key order
//        both operands share), so O^T[d][q] also lands in query fr's lane and
//        the rescale by exp(m_old - m_new) is one scalar per lane.
// Softmax in base 2 (scale * log2 e folded into the scores).  Causal: tiles past
// the block's last query are skipped, keys > query masked.
// ---------------------------------------------------------------------------
template <typename T, int HD>
__global__ __launch_bounds__(256, 2) void flash_attn_kernel(const T* __restrict__ qkv, T* __restrict__ out, int N,
                                                            int H, int D, int causal, float scale_log2) {
  typedef typename Vec8<T>::type V8;
  typedef typename Vec4<T>::type V4;
  typedef typename TrRead<T>::V4 TR4;
  constexpr int HK = (HD + 31) / 32 * 32, HV = (HD + 15) / 16 * 16;
  constexpr int KT = 64, QW = 32, QB = 4 * QW;  // keys per tile, queries per wave / block
  constexpr int CH = HD / 8;                    // 16-byte chunks per head row
  constexpr int KROW = HK * 2 + 16;             // K rows: an odd count of 16-byte slots
  constexpr int VROW = 160;                     // V rows: 40 banks, so the 8 rows one 32-lane
                                                // half of a transposed read touches are disjoint
  static_assert(HV * 2 <= VROW, "V row");
  constexpr int KBUF = KT * KROW, VBUF = KT * VROW, BUF = KBUF + VBUF;
  constexpr int PER = (KT * CH + 255) / 256;    // 16-byte chunks of K (and of V) per thread per tile
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nqb = (N + QB - 1) / QB;
  const int qb = blockIdx.x % nqb, bh = blockIdx.x / nqb;
  const int b = bh / H, h = bh % H;
  const long ld = 3L * D;
  const T* base = qkv + (long)b * N * ld + (long)h * HD;
  const int fr = lane & 15, fq = lane >> 4;

  // zero the padding that tile stores never write (both buffers): K cols HD..HK, V cols HD..HV
  if constexpr (HK > HD) {
    constexpr int PADC = HK / 8 - CH;
    for (int q = tid; q < 2 * KT * PADC; q += 256) {
      const int bf = q / (KT * PADC), r = (q / PADC) % KT, c = CH + q % PADC;
      *(V8*)(smem + bf * BUF + r * KROW + c * 16) = V8{};
    }
  }
  if constexpr (HV > HD) {
    constexpr int PADC = HV / 8 - CH;
    for (int q = tid; q < 2 * KT * PADC; q += 256) {
      const int bf = q / (KT * PADC), r = (q / PADC) % KT, c = CH + q % PADC;
      *(V8*)(smem + bf * BUF + KBUF + r * VROW + c * 16) = V8{};
    }
  }

  // this wave's 32 queries: Q fragments (B operand: [d][query]), head dim zero-padded to HK
  const int q0 = qb * QB + wave * QW;
  V8 qf[2][HK / 32];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const int qr = min(q0 + qi * 16 + fr, N - 1);
#pragma unroll
    for (int kk = 0; kk < HK / 32; ++kk) {
      const int c = kk * 4 + fq;
      qf[qi][kk] = c < CH ? *(const V8*)(base + (long)qr * ld + c * 8) : V8{};
    }
  }
  f32x4 o[2][HV / 16];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi)
#pragma unroll
    for (int ni = 0; ni < HV / 16; ++ni) o[qi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};

  // Two register sets of K/V chunks: while tile kt is computed from LDS buffer kt & 1,
  // set (kt + 1) & 1 holds tile kt + 1 (loads issued a tile earlier) and set kt & 1 takes
  // the loads of tile kt + 2 -- two tiles of latency cover.  The tile loop is unrolled by
  // two so every register-set index is static.
  V8 kr[2][PER], vr[2][PER];
  auto load_tile = [&](int kt, auto setc) {
    constexpr int S = decltype(setc)::value;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = tid + 256 * i, r = q / CH, c = q - r * CH, key = kt * KT + r;
      const bool ok = q < KT * CH && key < N;
      kr[S][i] = ok ? *(const V8*)(base + (long)key * ld + D + c * 8) : V8{};
      vr[S][i] = ok ? *(const V8*)(base + (long)key * ld + 2 * D + c * 8) : V8{};
    }
  };
  auto store_tile = [&](auto setc) {  // set S -> LDS buffer S
    constexpr int S = decltype(setc)::value;
    char* const sK = smem + S * BUF;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = tid + 256 * i, r = q / CH, c = q - r * CH;
      if (q < KT * CH) {
        *(V8*)(sK + r * KROW + c * 16) = kr[S][i];
        *(V8*)(sK + KBUF + r * VROW + c * 16) = vr[S][i];
      }
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;

  const int last_key = causal ? min(N, qb * QB + QB) : N;
  const int ntiles = (last_key + KT - 1) / KT;
  load_tile(0, S0{});
  store_tile(S0{});
  if (1 < ntiles) load_tile(1, S1{});
  __syncthreads();
  auto tile_step = [&](int kt, auto par) {
    constexpr int P = decltype(par)::value;  // == kt & 1
    using SP = std::integral_constant<int, P>;
    using SQ = std::integral_constant<int, 1 - P>;
    const char* const sK = smem + P * BUF;
    const char* const sV = sK + KBUF;
    if (kt + 2 < ntiles) load_tile(kt + 2, SP{});

    // S^T: s[qi][t][j] = S[query q0 + qi*16 + fr][key kt*64 + t*16 + 4fq + j]
    f32x4 s[2][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      V8 ka[HK / 32];
#pragma unroll
      for (int kk = 0; kk < HK / 32; ++kk) ka[kk] = *(const V8*)(sK + (t * 16 + fr) * KROW + (kk * 4 + fq) * 16);
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        s[qi][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < HK / 32; ++kk) s[qi][t] = mfma_16x16x32(ka[kk], qf[qi][kk], s[qi][t]);
      }
    }
    // online softmax: each lane holds one query (fr) per q-block.  Max in raw score
    // units (scale > 0), the scale folded into the exp2 argument (one FMA, raw v_exp_f32:
    // denormal results flush to 0); masks only on the tiles that need them (the ragged
    // last tile, causal tiles on the diagonal) -- a separate instantiation, so the common
    // tile carries no mask code.
    auto softmax = [&](auto masked) {
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        if constexpr (decltype(masked)::value) {
          const int qrow = q0 + qi * 16 + fr;
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int key = kt * KT + t * 16 + 4 * fq + j;
              if (key >= N || (causal && key > qrow)) s[qi][t][j] = -INFINITY;
            }
        }
        float mt = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) mt = fmaxf(mt, s[qi][t][j]);
        mt = xmax32(xmax16(mt));
        const float mn = fmaxf(m[qi], mt);
        const float corr = __builtin_amdgcn_exp2f((m[qi] - mn) * scale_log2);  // m = -inf first: 0
        const float off = -mn * scale_log2;
        float sum = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float e = __builtin_amdgcn_exp2f(fmaf(s[qi][t][j], scale_log2, off));
            s[qi][t][j] = e;
            sum += e;
          }
        // per-lane partial row sums (this lane's keys); the 4 lanes of a query are added
        // once after the last tile (corr is the same in all 4: the max is reduced per tile)
        l[qi] = l[qi] * corr + sum;
        m[qi] = mn;
#pragma unroll
        for (int ni = 0; ni < HV / 16; ++ni) o[qi][ni] *= corr;
      }
    };
    if (kt * KT + KT > N || (causal && kt * KT + KT - 1 > qb * QB)) softmax(std::true_type{});
    else softmax(std::false_type{});
    // O^T[d][q] += V^T P^T over 2 k-steps of 32 keys; k order (both operands):
    // element e of lane quarter fq <-> key 32ks + 16(e >> 2) + 4fq + (e & 3)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      V8 pf[2];
#pragma unroll
      for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int e = 0; e < 8; ++e) pf[qi][e] = (T)s[qi][2 * ks + (e >> 2)][e & 3];
      const char* const va0 = sV + (32 * ks + 4 * fq + (fr >> 2)) * VROW + 8 * (fr & 3);
#pragma unroll
      for (int ni = 0; ni < HV / 16; ++ni) {
        const TR4 lo = TrRead<T>::read(va0 + ni * 32);
        const TR4 hi = TrRead<T>::read(va0 + 16 * VROW + ni * 32);
        V8 va;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          va[e] = lo[e];
          va[e + 4] = hi[e];
        }
#pragma unroll
        for (int qi = 0; qi < 2; ++qi) o[qi][ni] = mfma_16x16x32(va, pf[qi], o[qi][ni]);
      }
    }
    if (kt + 1 < ntiles) store_tile(SQ{});
    __syncthreads();
  };
  for (int kt = 0; kt < ntiles; kt += 2) {
    tile_step(kt, S0{});
    if (kt + 1 < ntiles) tile_step(kt + 1, S1{});
  }
  // O^T[d = ni*16 + 4fq + j][q = fr]: 4 consecutive head dims per lane -> one 8-byte store
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const int q = q0 + qi * 16 + fr;
    const float lsum = xsum32(xsum16(l[qi]));  // all lanes (cross-lane), before the row mask
    if (q >= N) continue;
    const float inv = 1.0f / lsum;
    T* dst = out + ((long)b * N + q) * D + (long)h * HD;
#pragma unroll
    for (int ni = 0; ni < HV / 16; ++ni) {
      const int d0 = ni * 16 + 4 * fq;
      if (d0 < HD) {
        V4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (T)(o[qi][ni][j] * inv);
        *(V4*)(dst + d0) = w;
      }
    }
  }
}

template <typename T, int HD>
hipError_t launch_flash(const void* qkv, void* out, int B, int N, int H, int D, int causal, hipStream_t s) {
  const int nqb = (N + 127) / 128;
  hipLaunchKernelGGL((flash_attn_kernel<T, HD>), dim3(B * H * nqb), dim3(256), 0, s, (const T*)qkv, (T*)out, N, H, D,
                     causal, 1.4426950408889634f / sqrtf((float)HD));
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
// head): scores by threads over keys (16-byte K loads against the f32 query in LDS), block
// softmax, then o = sum_n p_n v_n with 16 key groups x 16 lanes of 8 head dims (16-byte V
// loads), the groups summed through LDS.  Memory-bound and tiny next to the trunk.
template <typename T>
__global__ __launch_bounds__(256) void map_attn_kernel(const float* __restrict__ q, const T* __restrict__ kv,
                                                       T* __restrict__ out, int N, int H, int D, float scale) {
  typedef typename Vec8<T>::type V8;
  __shared__ float sS[1024];
  __shared__ float sQ[128];
  __shared__ float sO[16][129];
  __shared__ float red[4];
  const int b = blockIdx.x / H, h = blockIdx.x % H, hd = D / H, ch = hd / 8;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* kvb = kv + (long)b * N * 2 * D + (long)h * hd;
  if (tid < hd) sQ[tid] = q[(long)h * hd + tid];
  __syncthreads();
  float lmax = -INFINITY;
  for (int n = tid; n < N; n += 256) {
    const T* kr = kvb + (long)n * 2 * D;
    float s = 0.f;
    for (int c = 0; c < ch; ++c) {
      const V8 k8 = *(const V8*)(kr + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) s = fmaf(sQ[c * 8 + e], (float)k8[e], s);
    }
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
  const int g = tid >> 4, c = tid & 15;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < ch) {
    for (int n = g; n < N; n += 16) {
      const V8 v8 = *(const V8*)(kvb + (long)n * 2 * D + D + c * 8);
      const float pn = sS[n];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(pn, (float)v8[e], acc[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) sO[g][c * 8 + e] = acc[e];
  }
  __syncthreads();
  if (tid < hd) {
    float o = 0.f;
#pragma unroll
    for (int gg = 0; gg < 16; ++gg) o += sO[gg][tid];
    out[(long)b * D + (long)h * hd + tid] = (T)(o * inv);
  }
}

}  // namespace

hipError_t launch_map_attention(DType dt, const float* q, const void* kv, void* out, int B, int N, int H, int D,
                                hipStream_t s) {
  if (B <= 0 || N <= 0 || N > 1024 || H <= 0 || D % H || D / H > 128 || (D / H) % 8) return hipErrorInvalidValue;
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
