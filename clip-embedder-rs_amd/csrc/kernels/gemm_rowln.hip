// Row-complete residual GEMM with the following LayerNorm fused in (gfx950):
//
//   x[m][:] += A[m][:] . W^T + bias          (out_proj / c_proj + residual, f32 residual stream)
//   h[m][:]  = LayerNorm(x[m][:]) * g + b    (ln_2 after out_proj, the next layer's ln_1 after c_proj)
//
// for the N = width GEMMs of the trunk (open_clip ResidualAttentionBlock, pull_onnx.py:53-68:
// x = x + attn(ln_1(x)); x = x + mlp(ln_2(x))).  A tile is 64 rows x ALL D columns, so the
// epilogue holds complete rows and the LayerNorm pass (ln_rows_kernel: read x, write h) over
// HBM disappears.  8 waves split the columns (D / 8 each); BK = 32 K-steps, staged by LDS-DMA
// into NS = 2..4 buffers (the DMA of step k + NS - 1 is issued when step k starts).
//
// The GEMM sums are the tiled kernels' sums bit for bit (same MFMA operand roles, K order and
// epilogue float ops: y = (acc + bias) + x), so the residual stream equals the unfused path's;
// the LayerNorm reduces in a different order than ln_rows_kernel (two-pass f32 mean / biased
// variance, torch semantics), so h differs from the unfused path in the last bits.
#include <algorithm>

#include <hip/hip_ext.h>

#include "common.hpp"
#include "gemm_util.hpp"
#include "kernels.hpp"

namespace clipgpu {

// Diagnostic build only (make stamps): s_memtime stamps of wave 0 of each block (slots: 0 start,
// 1 prologue issued, 2 + kt K-step kt done (kt < 40), 50 main loop done, 51 residual stored,
// 52 mean reduced, 53 variance reduced, 54 end; 62 / 63 realtime at start / end).
#ifdef CLIPGPU_GEMM_STAMPS
constexpr int kRlStampBlocks = 2048, kRlStampSlots = 64;
__device__ unsigned long long g_rowln_stamps[kRlStampBlocks * kRlStampSlots];
#define RL_STAMP(slot)                                                                          \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < kRlStampBlocks && (slot) < kRlStampSlots)               \
      g_rowln_stamps[blockIdx.x * kRlStampSlots + (slot)] = __builtin_amdgcn_s_memtime();       \
  } while (0)
#define RL_STAMP_REAL(slot)                                                                     \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < kRlStampBlocks)                                        \
      g_rowln_stamps[blockIdx.x * kRlStampSlots + (slot)] = __builtin_amdgcn_s_memrealtime();   \
  } while (0)
#else
#define RL_STAMP(slot) do {} while (0)
#define RL_STAMP_REAL(slot) do {} while (0)
#endif

namespace {

using namespace gemm_detail;

constexpr int RL_BM = 64;            // rows per tile
constexpr int RL_BK = 32;            // K per step (one MFMA K)
constexpr int RL_ROWB = RL_BK * 2;   // LDS bytes per staged row (64)
constexpr int RL_NW = 8;             // waves
constexpr int RL_SCRATCH = 4096;     // LN partial sums [8 waves][64 rows] f32 (+ spare)
constexpr int LDS_CAP = 160 * 1024;

template <int D>
struct RowLnCfg {
  static constexpr int CW = D / RL_NW;             // columns per wave
  static constexpr int NI = CW / 16;               // 16-column MFMA blocks per wave
  static constexpr int MI = RL_BM / 16;            // 16-row blocks
  static constexpr int PA = RL_BM / 16;            // DMA pieces of A per step (1 KiB = 16 rows x 64 B)
  static constexpr int PWt = D / 16;               // DMA pieces of W per step
  static constexpr int PT = PA + PWt;
  static constexpr int NP = (PT + RL_NW - 1) / RL_NW;   // pieces per wave (the first PT % NW waves)
  static constexpr int NP_LO = PT / RL_NW;               // the other waves
  static constexpr int EXTRA = PT % RL_NW;               // waves issuing NP pieces
  static constexpr int STAGE = (RL_BM + D) * RL_ROWB;
  static constexpr int NS = (LDS_CAP - RL_SCRATCH) / STAGE >= 4 ? 4 : (LDS_CAP - RL_SCRATCH) / STAGE;
  static_assert(D % 128 == 0 && NI >= 1 && NS >= 2, "unsupported width");
};

// XOR swizzle of the 16-byte chunk c (0..3) of LDS row r, conflict-free for the fragment reads
// (lane (fr, fq) reads row fr, chunk fq; ds_read_b128 lane groups {0-3,12-15,20-27}, ...): the
// 16 lanes of every group land on 16 distinct 16-byte slots of the 256-byte bank row.
__device__ __forceinline__ int rl_swz(int r, int c) { return c ^ ((0x1320 >> (((r >> 2) & 3) * 4)) & 3); }

template <int N>
__device__ __forceinline__ void rl_vm_wait_le() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N < 63 ? N : 63) : "memory");
}
// s_waitcnt vmcnt(n) for a wave-uniform runtime n <= 31
__device__ __forceinline__ void rl_vm_wait(int n) {
  switch (n) {
#define RL_CASE(k) case k: rl_vm_wait_le<k>(); break;
    RL_CASE(0) RL_CASE(1) RL_CASE(2) RL_CASE(3) RL_CASE(4) RL_CASE(5) RL_CASE(6) RL_CASE(7)
    RL_CASE(8) RL_CASE(9) RL_CASE(10) RL_CASE(11) RL_CASE(12) RL_CASE(13) RL_CASE(14) RL_CASE(15)
    RL_CASE(16) RL_CASE(17) RL_CASE(18) RL_CASE(19) RL_CASE(20) RL_CASE(21) RL_CASE(22) RL_CASE(23)
    RL_CASE(24) RL_CASE(25) RL_CASE(26) RL_CASE(27) RL_CASE(28) RL_CASE(29) RL_CASE(30)
#undef RL_CASE
    default: rl_vm_wait_le<0>(); break;
  }
}

template <typename T, int D>
__global__ __launch_bounds__(RL_NW * 64, 2) void gemm_rowln_kernel(RowLnParams p) {
  using C = RowLnCfg<D>;
  typedef typename Vec8<T>::type V8;
  typedef typename Vec4<T>::type V4;
  constexpr int NI = C::NI, MI = C::MI, CW = C::CW, NS = C::NS, STAGE = C::STAGE;
  constexpr int A_BYTES = RL_BM * RL_ROWB;
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE + RL_SCRATCH];

  RL_STAMP_REAL(62);
  RL_STAMP(0);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m0 = blockIdx.x * RL_BM;
  const int nk = p.K / RL_BK;
  const int my_np = wave < C::EXTRA || C::EXTRA == 0 ? C::NP : C::NP_LO;

  // ---- LDS-DMA: piece q (wave + 8 i) of a step: q < PA -> A rows 16q.., else W rows 16(q-PA)..;
  // lane l fills row (l >> 2) of the piece, 16-byte slot (l & 3), holding global chunk
  // rl_swz(row, slot) (the swizzle is an involution on the chunk index)
  uint32_t poff[C::NP];
  const char* const Ab = (const char*)p.A;
  const char* const Wb = (const char*)p.W;
#pragma unroll
  for (int i = 0; i < C::NP; ++i) {
    const int q = wave + RL_NW * i;
    const int rr = (q < C::PA ? q : q - C::PA) * 16 + (lane >> 2);
    const int c = rl_swz(rr, lane & 3);
    if (q >= C::PT) {
      poff[i] = 0;
    } else if (q < C::PA) {
      poff[i] = (uint32_t)((min(m0 + rr, p.M - 1) * (int)p.lda + c * 8) * 2);
    } else {
      poff[i] = (uint32_t)((rr * (int)p.ldw + c * 8) * 2);
    }
  }
  auto dma_step = [&](int kt) {
    char* const st = smem + (kt % NS) * STAGE;
#pragma unroll
    for (int i = 0; i < C::NP; ++i) {
      const int q = wave + RL_NW * i;
      if (q >= C::PT) break;
      if (q < C::PA) glds16(Ab + (size_t)kt * RL_ROWB + poff[i], st + q * 1024);
      else glds16(Wb + (size_t)kt * RL_ROWB + poff[i], st + A_BYTES + (q - C::PA) * 1024);
    }
  };

  // ---- fragments: lane (fr, fq) reads row fr of a 16-row block, K chunk fq (8 elements)
  const int fr = lane & 15, fq = lane >> 4;
  uint32_t offA[MI], offW[NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    const int r = mi * 16 + fr;
    offA[mi] = (uint32_t)(r * RL_ROWB + rl_swz(r, fq) * 16);
  }
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int r = wave * CW + ni * 16 + fr;
    offW[ni] = (uint32_t)(A_BYTES + r * RL_ROWB + rl_swz(r, fq) * 16);
  }
  const uint32_t lds0 = lds_addr(smem);

  f32x4 acc[NI][MI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) acc[ni][mi] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- L2 prefetch: the trunk's A and W are streamed once per launch, so every K-step's DMA
  // would pay HBM latency (several steps' worth: each step is only 64 B per row).  pfd steps
  // ahead (even steps: one 128-byte line covers two), wave 0 touches this tile's 64 A rows and
  // waves 1-2 two 64-row groups of W (the block's XCD-mates, blocks b + 8j, take the other
  // groups) with 4-byte LDS-DMA loads into a per-wave scratch slot: an L2 fill, no registers.
  constexpr int G = D / 64;
  const int pfd = p.pf;
  const int my_pf = pfd > 0 && wave <= 2 ? 1 : 0;
  uint32_t pf_off = 0;
  if (wave == 0) {
    pf_off = (uint32_t)(min(m0 + lane, p.M - 1) * (int)p.lda * 2);
  } else if (wave <= 2) {
    const int g = ((int)(blockIdx.x >> 3) + (wave - 1) * (G / 2)) % G;
    pf_off = (uint32_t)((g * 64 + lane) * (int)p.ldw * 2);
  }
  const char* const pf_base = wave == 0 ? Ab : Wb;
  char* const pf_slot = smem + NS * STAGE + RL_SCRATCH - (RL_NW - wave) * 256;
  auto pf_on = [&](int j) { return my_pf && j >= 0 && j + pfd < nk && ((j + pfd) & 1) == 0; };
  auto dma_n = [&](int s) { return s < nk ? my_np : 0; };
  // the epilogue's residual rows (64 x D f32 = XL lines of 128 B), touched at slot jx so that the
  // epilogue's loads hit L2: XN 4-byte DMA loads per wave, one line per lane
  constexpr int XLR = D * 4 / 128, XN = RL_BM * XLR / 64 / RL_NW;
  static_assert(RL_BM * XLR % (64 * RL_NW) == 0, "x prefetch split");
  const int jx = pfd > 0 ? max(0, nk - 4) : -1 << 20;
  auto x_on = [&](int j) { return j == jx ? XN : 0; };

  // prologue: steps 0 .. NS-2 in flight (issue slots j = 1-NS .. -1: DMA(j + NS - 1), no prefetch)
  for (int s = 0; s < NS - 1 && s < nk; ++s) dma_step(s);
  RL_STAMP(1);

  for (int kt = 0; kt < nk; ++kt) {
    // slot j issued DMA(j + NS - 1) then the prefetch of step j + pfd: DMA(kt) (slot kt-NS+1) has
    // landed once only the younger slots' loads are outstanding
    int younger = (pf_on(kt - NS + 1) ? 1 : 0) + x_on(kt - NS + 1);
#pragma unroll
    for (int j = kt - NS + 2; j <= kt - 1; ++j) younger += dma_n(j + NS - 1) + (pf_on(j) ? 1 : 0) + x_on(j);
    rl_vm_wait(younger);
    __builtin_amdgcn_s_barrier();  // every wave's pieces of step kt landed; step kt-1's buffer is free
    if (kt + NS - 1 < nk) dma_step(kt + NS - 1);
    if (pf_on(kt)) glds4(pf_base + (size_t)(kt + pfd) * RL_ROWB + pf_off, pf_slot);
    if (kt == jx) {
#pragma unroll
      for (int i = 0; i < XN; ++i) {
        const int L = (wave * XN + i) * 64 + lane;
        const int m = min(m0 + L / XLR, p.M - 1);
        glds4((const char*)p.x + ((size_t)m * D * 4 + (L % XLR) * 128), pf_slot);
      }
    }
    const uint32_t buf = lds0 + (kt % NS) * STAGE;
    V8 a[MI], w[NI];
    static_for<MI>([&](auto mi) { ds_read_b128<0>(a[mi], buf + offA[mi]); });
    static_for<NI>([&](auto ni) { ds_read_b128<0>(w[ni], buf + offW[ni]); });
    lgkm_wait_all(a, w);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) acc[ni][mi] = mfma_16x16x32(w[ni], a[mi], acc[ni][mi]);
    if (kt < 40) RL_STAMP(2 + kt);
  }
  RL_STAMP(50);

  // ---- epilogue: y = (acc + bias) + x -> x; LayerNorm(y) -> h ------------------------------
  // lane (fr, fq) owns rows mi*16 + fr and columns wave*CW + ni*16 + fq*4 .. +3
  // residual rows: all up front when registers allow (NI <= 6), else one 16-row block at a time
  constexpr bool XALL = NI <= 6;
  constexpr int XM = XALL ? MI : 1;
  float4 xr[XM][NI];
  auto load_x = [&](int mi, float4 (&dst)[NI]) {
    const int m = min(m0 + mi * 16 + fr, p.M - 1);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) dst[ni] = *(const float4*)(p.x + (long)m * D + wave * CW + ni * 16 + fq * 4);
  };
  if constexpr (XALL) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) load_x(mi, xr[mi]);
  }
  float4 bv[NI];
  if (p.bias) {
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) bv[ni] = *(const float4*)(p.bias + wave * CW + ni * 16 + fq * 4);
  } else {
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) bv[ni] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float s[MI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    s[mi] = 0.f;
    const int m = m0 + mi * 16 + fr;
    if constexpr (!XALL) load_x(mi, xr[0]);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int n = wave * CW + ni * 16 + fq * 4;
      const float4 b = bv[ni];
      const float4 xv = xr[XALL ? mi : 0][ni];
      f32x4 y;
      y[0] = (acc[ni][mi][0] + b.x) + xv.x;
      y[1] = (acc[ni][mi][1] + b.y) + xv.y;
      y[2] = (acc[ni][mi][2] + b.z) + xv.z;
      y[3] = (acc[ni][mi][3] + b.w) + xv.w;
      acc[ni][mi] = y;
      if (m < p.M) *(float4*)(p.x + (long)m * D + n) = make_float4(y[0], y[1], y[2], y[3]);
      s[mi] += (y[0] + y[1]) + (y[2] + y[3]);
    }
  }
  RL_STAMP(51);
  if (p.h == nullptr) {
    RL_STAMP_REAL(63);
    return;
  }
  // LN affine parameters of this lane's columns, loaded before the reductions (a wait for them
  // after the first h store would also wait for that store: vmcnt counts both in order)
  // (NI <= 6; wider tiles load them per use, registers being short)
  constexpr int GN = XALL ? NI : 1;
  float4 gv[GN], bbv[GN];
  if constexpr (XALL) {
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      gv[ni] = *(const float4*)(p.ln_w + wave * CW + ni * 16 + fq * 4);
      bbv[ni] = *(const float4*)(p.ln_b + wave * CW + ni * 16 + fq * 4);
    }
  }
  // LDS-only barrier: __syncthreads would also wait for this wave's residual stores
  auto lds_barrier = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  float* red = (float*)(smem + NS * STAGE);  // [8 waves][64 rows]
  // mean: per row, the 4 lanes (fq) of this wave, then the 8 waves
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    const float v = xsum32(xsum16(s[mi]));
    if (fq == 0) red[wave * RL_BM + mi * 16 + fr] = v;
  }
  lds_barrier();
  RL_STAMP(52);
  float mean[MI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < RL_NW; ++w) t += red[w * RL_BM + mi * 16 + fr];
    mean[mi] = t / (float)D;
  }
  lds_barrier();  // every wave read its means before the variance partials overwrite red
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    float q = 0.f;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const float a0 = acc[ni][mi][0] - mean[mi], a1 = acc[ni][mi][1] - mean[mi];
      const float a2 = acc[ni][mi][2] - mean[mi], a3 = acc[ni][mi][3] - mean[mi];
      q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
    q = xsum32(xsum16(q));
    if (fq == 0) red[wave * RL_BM + mi * 16 + fr] = q;
  }
  lds_barrier();
  RL_STAMP(53);
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < RL_NW; ++w) t += red[w * RL_BM + mi * 16 + fr];
    const float rstd = 1.0f / sqrtf(t / (float)D + p.eps);
    const int m = m0 + mi * 16 + fr;
    if (m >= p.M) continue;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int n = wave * CW + ni * 16 + fq * 4;
      const float4 g = XALL ? gv[XALL ? ni : 0] : *(const float4*)(p.ln_w + n);
      const float4 bb = XALL ? bbv[XALL ? ni : 0] : *(const float4*)(p.ln_b + n);
      V4 o;
      o[0] = (T)((acc[ni][mi][0] - mean[mi]) * rstd * g.x + bb.x);
      o[1] = (T)((acc[ni][mi][1] - mean[mi]) * rstd * g.y + bb.y);
      o[2] = (T)((acc[ni][mi][2] - mean[mi]) * rstd * g.z + bb.z);
      o[3] = (T)((acc[ni][mi][3] - mean[mi]) * rstd * g.w + bb.w);
      *(V4*)((T*)p.h + (long)m * D + n) = o;
    }
  }
  RL_STAMP(54);
  RL_STAMP_REAL(63);
}

template <typename T, int D>
hipError_t launch_rowln_t(const RowLnParams& p, hipStream_t s) {
  const int tiles = (p.M + RL_BM - 1) / RL_BM;
  gemm_launch(gemm_rowln_kernel<T, D>, tiles, RL_NW * 64, s, p);
  return hipGetLastError();
}

}  // namespace

bool gemm_rowln_supported(int D, int K) {
  return (D == 512 || D == 768 || D == 1024) && K % RL_BK == 0 && K > 0;
}

hipError_t launch_gemm_rowln(DType dt, const RowLnParams& p, hipStream_t s) {
  if (!gemm_rowln_supported(p.D, p.K) || p.M <= 0 || p.lda % 8 || p.ldw % 8) return hipErrorInvalidValue;
  if ((long)p.D * p.ldw * 2 >= (1L << 31)) return hipErrorInvalidValue;
  if (p.h != nullptr && (p.ln_w == nullptr || p.ln_b == nullptr)) return hipErrorInvalidValue;
  if ((long)p.M * p.lda * 2 >= (1L << 31)) {  // 32-bit per-lane staging offsets: row chunks (bit-invisible)
    long chunk = ((1L << 31) - 1) / (2 * p.lda);
    chunk -= chunk % 256;
    for (long m0 = 0; m0 < p.M; m0 += chunk) {
      RowLnParams q = p;
      q.M = (int)std::min<long>(chunk, p.M - m0);
      q.A = (const char*)p.A + m0 * p.lda * 2;
      q.x = p.x + m0 * p.D;
      if (p.h) q.h = (char*)p.h + m0 * p.D * 2;
      const hipError_t err = launch_gemm_rowln(dt, q, s);
      if (err != hipSuccess) return err;
    }
    return hipSuccess;
  }
  switch (p.D) {
    case 512: return dt == DT_BF16 ? launch_rowln_t<__bf16, 512>(p, s) : launch_rowln_t<_Float16, 512>(p, s);
    case 768: return dt == DT_BF16 ? launch_rowln_t<__bf16, 768>(p, s) : launch_rowln_t<_Float16, 768>(p, s);
    default: return dt == DT_BF16 ? launch_rowln_t<__bf16, 1024>(p, s) : launch_rowln_t<_Float16, 1024>(p, s);
  }
}

#ifdef CLIPGPU_GEMM_STAMPS
hipError_t read_rowln_stamps(unsigned long long* host, int nblocks, bool clear) {
  const size_t n = (size_t)std::min(nblocks, kRlStampBlocks) * kRlStampSlots * sizeof(unsigned long long);
  if (clear) {
    static unsigned long long zeros[kRlStampBlocks * kRlStampSlots];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_rowln_stamps), zeros, sizeof(zeros));
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rowln_stamps), n);
}
#endif

}  // namespace clipgpu
