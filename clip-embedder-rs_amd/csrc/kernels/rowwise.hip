// Row-wise (one wave per row) kernels: LayerNorm variants, token / patch
// stems, pooling and L2 normalisation.  All HBM-bound: float4 loads, the row
// held in registers, two-pass mean/variance in f32 (torch LayerNorm:
// (x - mean) / sqrt(var + eps) * w + b, biased variance).
//
// Reference semantics (graph content from pull_onnx.py:53-68, open_clip):
//   vision stem: x = [cls; conv1(x)] + pos; x = ln_pre(x)          (a10)
//   text stem:   x = token_embedding[ids] + positional_embedding    (a16)
//   tails:       ln_post(x[:,0]) / ln_final(x[b, argmax(ids[b])])    (a13, a18)
//   F.normalize: x / max(||x||_2, 1e-12)
#include <type_traits>

#include "common.hpp"
#include "kernels.hpp"

namespace clipgpu {

namespace {

constexpr int MAXV = 5;  // float4 per lane -> D <= 1280

// A row in registers: NV float4 per lane (lane-strided, float4 c = i*64 + lane); only the
// last of them can fall past D/4.  Kernels are instantiated per NV = ceil(D / 256).
template <int NV>
struct Row {
  float4 v[NV];
};

template <int NV>
__device__ __forceinline__ bool in_row(int i, int lane, int D4) {
  return i + 1 < NV || i * 64 + lane < D4;
}

template <int NV>
__device__ __forceinline__ void load_row(const float* src, int D4, int lane, Row<NV>& r) {
#pragma unroll
  for (int i = 0; i < NV; ++i)
    r.v[i] = in_row<NV>(i, lane, D4) ? ((const float4*)src)[i * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
}

// A residual-stream row stored as f16 (clipgpu_options.residual: 4 halves per lane slot, 8-byte
// accesses); the values are widened to f32 for every add and statistic.
typedef _Float16 Half4 __attribute__((ext_vector_type(4)));
template <int NV>
__device__ __forceinline__ void load_row(const _Float16* src, int D4, int lane, Row<NV>& r) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (in_row<NV>(i, lane, D4)) {
      const Half4 h = ((const Half4*)src)[i * 64 + lane];
      r.v[i] = make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
    } else {
      r.v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// torch LayerNorm statistics: two-pass mean / biased variance in f32, rstd = 1 / sqrt(var + eps).
template <int NV>
__device__ __forceinline__ void ln_stats_regs(const Row<NV>& in, float eps, int D, int lane, float& mean_out,
                                              float& rstd_out) {
  const int D4 = D >> 2;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += in.v[i].x + in.v[i].y + in.v[i].z + in.v[i].w;  // padding holds 0
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (in_row<NV>(i, lane, D4)) {
      const float a = in.v[i].x - mean, bb = in.v[i].y - mean, cc = in.v[i].z - mean, d = in.v[i].w - mean;
      q += a * a + bb * bb + cc * cc + d * d;
    }
  }
  const float var = wave_sum(q) / (float)D;
  mean_out = mean;
  rstd_out = 1.0f / sqrtf(var + eps);
}

// torch LayerNorm (ln_stats_regs, then the affine map); g, b preloaded rows.
template <int NV>
__device__ __forceinline__ void layer_norm_regs(const Row<NV>& in, Row<NV>& out, const Row<NV>& g, const Row<NV>& b,
                                                float eps, int D, int lane) {
  float mean, rstd;
  ln_stats_regs(in, eps, D, lane, mean, rstd);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    out.v[i].x = (in.v[i].x - mean) * rstd * g.v[i].x + b.v[i].x;
    out.v[i].y = (in.v[i].y - mean) * rstd * g.v[i].y + b.v[i].y;
    out.v[i].z = (in.v[i].z - mean) * rstd * g.v[i].z + b.v[i].z;
    out.v[i].w = (in.v[i].w - mean) * rstd * g.v[i].w + b.v[i].w;
  }
}

template <typename T, int NV>
__device__ __forceinline__ void store_row16(T* dst, const Row<NV>& r, int D4, int lane) {
  typedef typename Vec4<T>::type V4;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (in_row<NV>(i, lane, D4)) {
      V4 o;
      o[0] = (T)r.v[i].x; o[1] = (T)r.v[i].y; o[2] = (T)r.v[i].z; o[3] = (T)r.v[i].w;
      ((V4*)dst)[i * 64 + lane] = o;
    }
  }
}

// MX-fp8 row (gemm_mx.hip's A operand): e4m3 bytes + one E8M0 scale per 32 columns.  A
// 32-column block is 8 consecutive float4 = 8 consecutive lanes of one slot i; D % 32 == 0,
// so a block is wholly inside or outside the row.
template <int NV>
__device__ __forceinline__ void store_row_mx(uint8_t* q, uint8_t* qs, const Row<NV>& r, int D4, int lane) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float4 v = r.v[i];
    float amax = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
    amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
    amax = fmaxf(amax, __shfl_xor(amax, 4, 64));
    if (in_row<NV>(i, lane, D4)) {
      const int e = mx_exp(amax);
      const int c = i * 64 + lane;
      ((uint32_t*)q)[c] = mx_pack4(v.x, v.y, v.z, v.w, mx_inv(e));
      if ((lane & 7) == 0) qs[c >> 3] = (uint8_t)(e + 127);
    }
  }
}

// LayerNorm output: 16-bit row, or MX-fp8 (out = e4m3 bytes) when qs != nullptr.
template <typename T, int NV>
__device__ __forceinline__ void store_ln_out(T* out, uint8_t* qs, long row, int D, const Row<NV>& r, int lane) {
  if (qs != nullptr) store_row_mx((uint8_t*)out + row * D, qs + row * (D >> 5), r, D >> 2, lane);
  else store_row16(out + row * D, r, D >> 2, lane);
}

template <int NV>
__device__ __forceinline__ void store_row32(float* dst, const Row<NV>& r, int D4, int lane) {
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (in_row<NV>(i, lane, D4)) ((float4*)dst)[i * 64 + lane] = r.v[i];
}
// The residual row as the stream stores it (f16: every value rounded to f16, held as f32).
template <typename XT, int NV>
__device__ __forceinline__ void round_rowx(Row<NV>& r) {
  if constexpr (!std::is_same<XT, float>::value) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      r.v[i].x = (float)(_Float16)r.v[i].x; r.v[i].y = (float)(_Float16)r.v[i].y;
      r.v[i].z = (float)(_Float16)r.v[i].z; r.v[i].w = (float)(_Float16)r.v[i].w;
    }
  }
}
// residual-stream row store: f32, or rounded to f16
template <int NV>
__device__ __forceinline__ void store_rowx(float* dst, const Row<NV>& r, int D4, int lane) {
  store_row32(dst, r, D4, lane);
}
template <int NV>
__device__ __forceinline__ void store_rowx(_Float16* dst, const Row<NV>& r, int D4, int lane) {
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (in_row<NV>(i, lane, D4)) {
      Half4 h;
      h[0] = (_Float16)r.v[i].x; h[1] = (_Float16)r.v[i].y; h[2] = (_Float16)r.v[i].z; h[3] = (_Float16)r.v[i].w;
      ((Half4*)dst)[i * 64 + lane] = h;
    }
}

template <int NV>
__device__ __forceinline__ void add_row(Row<NV>& r, const Row<NV>& a) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    r.v[i].x += a.v[i].x; r.v[i].y += a.v[i].y; r.v[i].z += a.v[i].z; r.v[i].w += a.v[i].w;
  }
}

// Every kernel issues all of its row loads (activations and LN parameters) up front, so
// their latencies overlap instead of following the reductions one round trip at a time.

template <typename T, int NV, typename XT>
__global__ __launch_bounds__(256) void ln_rows_kernel(const XT* __restrict__ x, const float* w, const float* b,
                                                      float eps,
                                                      T* __restrict__ out, uint8_t* __restrict__ qs, int rows,
                                                      int D) {
  // one wave per row, rows strided by the grid's wave count (grid <= rows / 4 blocks); the next
  // row's loads are issued before this row's reductions, so a wave keeps two rows in flight
  const int stride = gridDim.x * 4, lane = threadIdx.x & 63;
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int D4 = D >> 2;
  Row<NV> r, g, bb;
  load_row(x + (long)row * D, D4, lane, r);
  load_row(w, D4, lane, g);
  load_row(b, D4, lane, bb);
  for (;;) {
    const int next = row + stride;
    Row<NV> nr;
    if (next < rows) load_row(x + (long)next * D, D4, lane, nr);
    Row<NV> o;
    layer_norm_regs(r, o, g, bb, eps, D, lane);
    store_ln_out(out, qs, row, D, o, lane);
    if (next >= rows) break;
    row = next;
    r = nr;
  }
}

// Row statistics only (the LayerNorm-folded GEMMs' GemmParams.rowstats): one wave per row as
// ln_rows_kernel, stats[row] = (mean, rstd) by the same arithmetic.  (T unused: the launch macro's.)
template <typename T, int NV, typename XT>
__global__ __launch_bounds__(256) void ln_stats_kernel(const XT* __restrict__ x, float eps, float* __restrict__ stats,
                                                       int rows, int D) {
  const int stride = gridDim.x * 4, lane = threadIdx.x & 63;
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int D4 = D >> 2;
  Row<NV> r;
  load_row(x + (long)row * D, D4, lane, r);
  for (;;) {
    const int next = row + stride;
    Row<NV> nr;
    if (next < rows) load_row(x + (long)next * D, D4, lane, nr);
    float mean, rstd;
    ln_stats_regs(r, eps, D, lane, mean, rstd);
    if (lane == 0) *(float2*)(stats + 2L * row) = make_float2(mean, rstd);
    if (next >= rows) break;
    row = next;
    r = nr;
  }
}

template <typename T, int NV, typename XT>
__global__ __launch_bounds__(256) void vision_embed_ln_kernel(XT* __restrict__ x, const float* cls,
                                                              const float* pos, const float* lnpre_w,
                                                              const float* lnpre_b, const float* ln1_w,
                                                              const float* ln1_b, float eps, T* __restrict__ h,
                                                              uint8_t* __restrict__ qs, int rows, int tokens, int D,
                                                              float* __restrict__ stats) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int D4 = D >> 2;
  Row<NV> r, y, z, g0, b0, g1, b1;
  if (row % tokens == 0) {  // CLS token: class_embedding + positional_embedding[0]
    Row<NV> c, p;
    load_row(cls, D4, lane, c);
    load_row(pos, D4, lane, p);
    r = c;
    add_row(r, p);
  } else {  // patch rows: conv1 + pos already written by the patch GEMM epilogue
    load_row(x + (long)row * D, D4, lane, r);
  }
  load_row(lnpre_w, D4, lane, g0);
  load_row(lnpre_b, D4, lane, b0);
  if (h != nullptr) {
    load_row(ln1_w, D4, lane, g1);
    load_row(ln1_b, D4, lane, b1);
  }
  layer_norm_regs(r, y, g0, b0, eps, D, lane);
  round_rowx<XT>(y);  // ln_1 of the residual row as stored
  store_rowx(x + (long)row * D, y, D4, lane);
  if (h == nullptr) {  // LayerNorm folded into the QKV GEMM: ln_1's statistics only
    float mean, rstd;
    ln_stats_regs(y, eps, D, lane, mean, rstd);
    if (lane == 0) *(float2*)(stats + 2L * row) = make_float2(mean, rstd);
    return;
  }
  layer_norm_regs(y, z, g1, b1, eps, D, lane);
  store_ln_out(h, qs, row, D, z, lane);
}

template <typename T, int NV, typename XT>
__global__ __launch_bounds__(256) void text_embed_ln_kernel(const int64_t* __restrict__ ids, const float* tok,
                                                            const float* pos, const float* ln1_w,
                                                            const float* ln1_b, float eps, XT* __restrict__ x,
                                                            T* __restrict__ h, uint8_t* __restrict__ qs, int rows,
                                                            int Tctx, int D, int vocab, float* __restrict__ stats) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int D4 = D >> 2;
  long id = ids[row];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);  // host validates; clamp keeps the gather in bounds
  Row<NV> e, p, y, g, bb;
  load_row(tok + id * D, D4, lane, e);
  load_row(pos + (long)(row % Tctx) * D, D4, lane, p);
  if (h != nullptr) {
    load_row(ln1_w, D4, lane, g);
    load_row(ln1_b, D4, lane, bb);
  }
  add_row(e, p);
  round_rowx<XT>(e);  // ln_1 of the residual row as stored
  store_rowx(x + (long)row * D, e, D4, lane);
  if (h == nullptr) {  // LayerNorm folded into the QKV GEMM: ln_1's statistics only
    float mean, rstd;
    ln_stats_regs(e, eps, D, lane, mean, rstd);
    if (lane == 0) *(float2*)(stats + 2L * row) = make_float2(mean, rstd);
    return;
  }
  layer_norm_regs(e, y, g, bb, eps, D, lane);
  store_ln_out(h, qs, row, D, y, lane);
}

// Token pooled for sequence bi: 0 (CLS, ids == nullptr) or the first index of the maximum
// id (torch argmax; EOT is the largest id).  Wave-uniform.
__device__ inline int pooled_token(const int64_t* __restrict__ ids, int bi, int tokens, int lane) {
  if (ids == nullptr) return 0;
  long best = -1;
  int bidx = 0x7fffffff;
  for (int t = lane; t < tokens; t += 64) {
    const long v = ids[(long)bi * tokens + t];
    if (v > best) { best = v; bidx = t; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const long ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bidx, o, 64);
    if (ov > best || (ov == best && oi < bidx)) { best = ov; bidx = oi; }
  }
  return bidx;
}

template <typename T, int NV, typename XT>
__global__ __launch_bounds__(256) void pool_ln_kernel(const XT* __restrict__ x,
                                                      const int64_t* __restrict__ ids, int tokens, const float* w,
                                                      const float* b, float eps, T* __restrict__ out, int B, int D) {
  const int bi = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (bi >= B) return;
  const int D4 = D >> 2;
  const int src = pooled_token(ids, bi, tokens, lane);
  Row<NV> r, y, g, bb;
  load_row(x + ((long)bi * tokens + src) * D, D4, lane, r);
  load_row(w, D4, lane, g);
  load_row(b, D4, lane, bb);
  layer_norm_regs(r, y, g, bb, eps, D, lane);
  store_row16(out + (long)bi * D, y, D4, lane);
}

// Last-layer compaction: the pooled token's residual row x and attention-output row h
// (16-bit, raw bits) of each sequence, copied to row bi of xc / hc.  One wave per sequence.
__global__ __launch_bounds__(256) void gather_pooled_kernel(const char* __restrict__ x,
                                                            const uint16_t* __restrict__ h,
                                                            const int64_t* __restrict__ ids, int tokens,
                                                            char* __restrict__ xc, uint16_t* __restrict__ hc, int B,
                                                            int D, int xbytes) {
  const int bi = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (bi >= B) return;
  const long src = (long)bi * tokens + pooled_token(ids, bi, tokens, lane);
  const long rb = (long)D * xbytes;  // residual row bytes (f32 or f16), a multiple of 8
  const uint2* xs = (const uint2*)(x + src * rb);
  uint2* xd = (uint2*)(xc + (long)bi * rb);
  for (int i = lane; i < rb / 8; i += 64) xd[i] = xs[i];
  const uint2* hs = (const uint2*)(h + src * D);
  uint2* hd = (uint2*)(hc + (long)bi * D);
  for (int i = lane; i < D / 4; i += 64) hd[i] = hs[i];
}

__global__ __launch_bounds__(256) void l2norm_kernel(const float* __restrict__ in, float* __restrict__ out, int B,
                                                     int E) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B) return;
  const float* src = in + (long)row * E;
  float s = 0.f;
  for (int c = lane; c < E; c += 64) s += src[c] * src[c];
  const float n = fmaxf(sqrtf(wave_sum(s)), 1e-12f);
  for (int c = lane; c < E; c += 64) out[(long)row * E + c] = src[c] / n;
}

template <typename T>
__global__ void cast_kernel(const float* __restrict__ in, T* __restrict__ out, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (T)in[i];
}

inline dim3 rows_grid(int rows) { return dim3((rows + 3) / 4); }

}  // namespace

// NV = ceil(D / 256) float4 per lane; D % 4 == 0, D <= 1280.
// KERNEL<T, NV, XT>: XT the residual-stream element type (float or _Float16).
#define CLIPGPU_ROW_LAUNCH_X(KERNEL, T, XT, GRID, D, ...)                                              \
  do {                                                                                                  \
    const int nv_ = ((D) / 4 + 63) / 64;                                                                \
    auto go_ = [&](auto nvc) {                                                                          \
      constexpr int NVC = decltype(nvc)::value;                                                         \
      hipLaunchKernelGGL((KERNEL<T, NVC, XT>), GRID, dim3(256), 0, s, __VA_ARGS__);                     \
    };                                                                                                  \
    switch (nv_) {                                                                                      \
      case 1: go_(std::integral_constant<int, 1>{}); break;                                             \
      case 2: go_(std::integral_constant<int, 2>{}); break;                                             \
      case 3: go_(std::integral_constant<int, 3>{}); break;                                             \
      case 4: go_(std::integral_constant<int, 4>{}); break;                                             \
      default: go_(std::integral_constant<int, 5>{}); break;                                            \
    }                                                                                                   \
  } while (0)
// f(T*, XT*) with T the 16-bit type of dt and XT the residual-stream type (x16: _Float16, else float):
// the four instantiations of a row kernel that touches the residual stream.
template <typename F>
inline void dispatch_dx(DType dt, int x16, F f) {
  if (dt == DT_BF16) {
    if (x16) f((__bf16*)nullptr, (_Float16*)nullptr);
    else f((__bf16*)nullptr, (float*)nullptr);
  } else {
    if (x16) f((_Float16*)nullptr, (_Float16*)nullptr);
    else f((_Float16*)nullptr, (float*)nullptr);
  }
}
#define CLIPGPU_TX_TYPES                                  \
  using T = std::remove_pointer_t<decltype(tp_)>;          \
  using XT = std::remove_pointer_t<decltype(xp_)>;         \
  (void)tp_;                                              \
  (void)xp_

// (16-bit output pointers are passed as void*: the kernel parameter is T*)
hipError_t launch_ln_rows(DType dt, const void* x, int x16, const float* w, const float* b, float eps, void* out16,
                          int rows, int D, hipStream_t s, uint8_t* qs) {
  if (D % 4 || D > 256 * MAXV || D <= 0 || (qs != nullptr && D % 32)) return hipErrorInvalidValue;
  // blocks: one row per wave, at most one resident round (8 blocks of 4 waves per CU); more rows
  // loop with the next row's loads in flight.  Measured against one row per wave at 12800 rows
  // (ViT-B/32, B = 256): 23 LayerNorms 263-266 vs 268-271 us per step serialized; 1600 / 800
  // blocks 272-276 / 295-297 us (profiles/r03_v9_ln_grid_ab.txt); bit-identical at every grid.
  dim3 grid = rows_grid(rows);
  const int cap = device_cus() * 8;
  if ((int)grid.x > cap) grid.x = cap;
  dispatch_dx(dt, x16, [&](auto tp_, auto xp_) {
    CLIPGPU_TX_TYPES;
    CLIPGPU_ROW_LAUNCH_X(ln_rows_kernel, T, XT, grid, D, (const XT*)x, w, b, eps, (T*)out16, qs, rows, D);
  });
  return hipGetLastError();
}

hipError_t launch_ln_stats(const void* x, int x16, float eps, float* stats, int rows, int D, hipStream_t s) {
  if (D % 4 || D > 256 * MAXV || D <= 0 || rows <= 0 || stats == nullptr) return hipErrorInvalidValue;
  dim3 grid = rows_grid(rows);
  const int cap = device_cus() * 8;
  if ((int)grid.x > cap) grid.x = cap;
  dispatch_dx(DT_BF16, x16, [&](auto tp_, auto xp_) {
    CLIPGPU_TX_TYPES;
    CLIPGPU_ROW_LAUNCH_X(ln_stats_kernel, T, XT, grid, D, (const XT*)x, eps, stats, rows, D);
  });
  return hipGetLastError();
}

hipError_t launch_vision_embed_ln(DType dt, void* x, int x16, const float* cls, const float* pos, const float* lnpre_w,
                                  const float* lnpre_b, const float* ln1_w, const float* ln1_b, float eps,
                                  void* h, int B, int tokens, int D, hipStream_t s, uint8_t* qs, float* stats) {
  if (h == nullptr && stats == nullptr) return hipErrorInvalidValue;
  if (D % 4 || D > 256 * MAXV || D <= 0 || (qs != nullptr && D % 32)) return hipErrorInvalidValue;
  const int rows = B * tokens;
  dispatch_dx(dt, x16, [&](auto tp_, auto xp_) {
    CLIPGPU_TX_TYPES;
    CLIPGPU_ROW_LAUNCH_X(vision_embed_ln_kernel, T, XT, rows_grid(rows), D, (XT*)x, cls, pos, lnpre_w, lnpre_b, ln1_w,
                         ln1_b, eps, (T*)h, qs, rows, tokens, D, stats);
  });
  return hipGetLastError();
}

hipError_t launch_text_embed_ln(DType dt, const int64_t* ids, const float* tok, const float* pos,
                                const float* ln1_w, const float* ln1_b, float eps, void* x, int x16, void* h,
                                int B, int Tctx, int D, int vocab, hipStream_t s, uint8_t* qs, float* stats) {
  if (h == nullptr && stats == nullptr) return hipErrorInvalidValue;
  if (D % 4 || D > 256 * MAXV || D <= 0 || (qs != nullptr && D % 32)) return hipErrorInvalidValue;
  const int rows = B * Tctx;
  dispatch_dx(dt, x16, [&](auto tp_, auto xp_) {
    CLIPGPU_TX_TYPES;
    CLIPGPU_ROW_LAUNCH_X(text_embed_ln_kernel, T, XT, rows_grid(rows), D, ids, tok, pos, ln1_w, ln1_b, eps, (XT*)x,
                         (T*)h, qs, rows, Tctx, D, vocab, stats);
  });
  return hipGetLastError();
}

hipError_t launch_gather_pooled(const void* x, int x16, const void* h16, const int64_t* ids, int tokens, void* xc,
                                void* hc16, int B, int D, hipStream_t s) {
  if (D % 4 || D <= 0 || B <= 0 || tokens <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_pooled_kernel, rows_grid(B), dim3(256), 0, s, (const char*)x, (const uint16_t*)h16, ids,
                     tokens, (char*)xc, (uint16_t*)hc16, B, D, x16 ? 2 : 4);
  return hipGetLastError();
}

hipError_t launch_pool_ln(DType dt, const void* x, int x16, const int64_t* ids, int tokens,
                          const float* w, const float* b, float eps, void* out16, int B, int D, hipStream_t s) {
  if (D % 4 || D > 256 * MAXV || D <= 0) return hipErrorInvalidValue;
  dispatch_dx(dt, x16, [&](auto tp_, auto xp_) {
    CLIPGPU_TX_TYPES;
    CLIPGPU_ROW_LAUNCH_X(pool_ln_kernel, T, XT, rows_grid(B), D, (const XT*)x, ids, tokens, w, b, eps, (T*)out16, B, D);
  });
  return hipGetLastError();
}

hipError_t launch_l2norm(const float* in, float* out, int B, int E, hipStream_t s) {
  hipLaunchKernelGGL(l2norm_kernel, rows_grid(B), dim3(256), 0, s, in, out, B, E);
  return hipGetLastError();
}

// Pull copy of a host-mapped (registered) range into device memory: every lane moves 16-byte
// chunks, grid-stride, so many CUs keep PCIe reads in flight (the host path's alternative to an
// SDMA H2D; clipgpu_test_host_plan copy_stream 3).  src / dst 16-byte aligned, bytes % 16 == 0.
__global__ __launch_bounds__(256) void pull_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        long n16) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) dst[i] = src[i];
}

hipError_t launch_pull_copy(const void* src_mapped, void* dst, size_t bytes, hipStream_t s) {
  if (((uintptr_t)src_mapped | (uintptr_t)dst | bytes) & 15) return hipErrorInvalidValue;
  const long n16 = (long)(bytes / 16);
  const long blocks = (n16 + 255) / 256 < 2048 ? (n16 + 255) / 256 : 2048;
  if (n16 == 0) return hipSuccess;
  hipLaunchKernelGGL(pull_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint4*)src_mapped, (uint4*)dst,
                     n16);
  return hipGetLastError();
}

hipError_t launch_cast_f32(DType dt, const float* in, void* out, long n, hipStream_t s) {
  const long blocks = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(cast_kernel<__bf16>, dim3((unsigned)blocks), dim3(256), 0, s, in, (__bf16*)out, n);
  else
    hipLaunchKernelGGL(cast_kernel<_Float16>, dim3((unsigned)blocks), dim3(256), 0, s, in, (_Float16*)out, n);
  return hipGetLastError();
}

}  // namespace clipgpu
