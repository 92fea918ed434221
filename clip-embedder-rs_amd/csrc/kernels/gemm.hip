// MFMA GEMM for the transformer towers, gfx950.
//
//   C[M][N] = A[M][K] . W[N][K]^T  (+ fused epilogue)
//
// Replaces the MatMul/Gemm/Conv nodes ONNX Runtime executes for the exported
// graphs (pull_onnx.py:53-68 -> src/vision.rs:108, src/text.rs:158-160):
// QKV in_proj, out_proj, c_fc (+activation), c_proj (+residual), the conv1
// patch embedding and the final projection.
//
// The patch-embedding conv runs as a row GEMM over the patch rows staged by
// launch_patch_rows (patch.hip), with the EPI_PATCH epilogue.
//
// Two kernels (GemmTile, kernels.hpp):
//   gemm_pipe_kernel    software-pipelined persistent tiles (K >= 128): 160x128, 256x128, 256x256,
//                       192x256, 224x192 (4 or 8 waves), LDS-DMA staged, 2 or 3 LDS stages
//   gemm_skinny_kernel  one wave per 16x16 output block, operands streamed from L2: M <= 256
//                       (the pruned last layer, the heads), and in its general form every shape
//                       the pipelined kernel does not take (K = 64, unaligned 16-bit rows)
// Each wave issues v_mfma_f32_16x16x32_{bf16,f16} (f32 accumulate).  Operand
// tiles (BK = 64) are staged global->LDS by global_load_lds_dwordx4 into a
// lane-linear image with the XOR swizzle applied on the SOURCE address and on
// the ds_read_b128 address (cdna_hip_programming.md §5.4 rule 21).  Block ids are
// remapped XCD-aware, then grouped row-panels at a time for L2 reuse.  Persistent:
// the grid is the resident block count and each block walks its tiles.  MFMA
// operands are swapped so each lane owns consecutive output columns (16-byte
// epilogue stores).  M and N tails: clamped source rows + masked stores; K must
// be a multiple of 64.  Every kernel and tile runs the same MFMA chain per output
// element in the same K order with the same epilogue float ops, so the tile choice
// never changes the bits.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include <hip/hip_ext.h>

#include "common.hpp"
#include "kernels.hpp"
#include "gemm_util.hpp"

namespace clipgpu {

thread_local GemmLaunchEvents g_gemm_events;

// Diagnostic build only (make stamps -> lib/libclipgpu_stamps.so): s_memtime
// stamps of wave 0 of each block at fixed points of the tile loop
// (tools/gemm_stamps.py).  The product build compiles them out.
#ifdef CLIPGPU_GEMM_STAMPS
constexpr int kStampBlocks = 2048, kStampSlots = 64;
__device__ unsigned long long g_gemm_stamps[kStampBlocks * kStampSlots];
#define GEMM_STAMP(slot)                                                                        \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks && (slot) < kStampSlots)                   \
      g_gemm_stamps[blockIdx.x * kStampSlots + (slot)] = __builtin_amdgcn_s_memtime();        \
  } while (0)
#define GEMM_STAMP_REAL(slot)                                                                   \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks)                                          \
      g_gemm_stamps[blockIdx.x * kStampSlots + (slot)] = __builtin_amdgcn_s_memrealtime();    \
  } while (0)
// slot 61: where the block runs, (XCC_ID << 32) | HW_ID (cu_id bits 11:8, sh 12, se 15:13)
#define GEMM_STAMP_HWID()                                                                       \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks)                                          \
      g_gemm_stamps[blockIdx.x * kStampSlots + 61] =                                            \
          ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |              \
          (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);                                  \
  } while (0)
#else
#define GEMM_STAMP(slot) do {} while (0)
#define GEMM_STAMP_REAL(slot) do {} while (0)
#define GEMM_STAMP_HWID() do {} while (0)
#endif

namespace {

#if CLIPGPU_GEMM_POISON
// (race-check build) NaN bytes over the 1 KiB an LDS-DMA of this wave is about to fill; the
// store is complete before the DMA is issued
__device__ __forceinline__ void poison_lds(char* dst) { gemm_detail::lds_poison_piece(dst); }
#define GEMM_POISON(dst) poison_lds(dst)
#else
#define GEMM_POISON(dst) do {} while (0)
#endif

using namespace gemm_detail;

constexpr int BK = 64;

// Race-check build (make poison -> lib/libclipgpu_poison.so, tests/test_gpu_kernels.py): before
// each LDS-DMA of the pipelined kernel, the issuing wave fills the destination with NaN bytes, so
// a fragment read that runs ahead of its DMA (a missing vmcnt wait or barrier) reads NaN instead
// of a stale but finite tile, and the result is no longer bit-identical to the product build's.
#ifndef CLIPGPU_GEMM_POISON
#define CLIPGPU_GEMM_POISON 0
#endif
#ifndef CLIPGPU_GEMM_SPREAD_W8
#define CLIPGPU_GEMM_SPREAD_W8 0
#endif
#ifndef CLIPGPU_GEMM_SPREAD_ALL
#define CLIPGPU_GEMM_SPREAD_ALL 0
#endif
#ifndef CLIPGPU_GEMM_NONPERSIST
#define CLIPGPU_GEMM_NONPERSIST 0
#endif
#ifndef CLIPGPU_GEMM_EPI_DMA_WAIT
#define CLIPGPU_GEMM_EPI_DMA_WAIT 1
#endif

template <typename T>
__device__ __forceinline__ T to16(float v) { return (T)v; }
__device__ __forceinline__ float4 widen4(float4 v) { return v; }
__device__ __forceinline__ float4 widen4(f16x4 h) { return make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]); }

// ---------------------------------------------------------------------------
// Software-pipelined GEMM for row-major A (the trunk GEMMs; K >= 128).
//
// Each 64-deep K-step g is two MFMA phases (kk0 = k 0..31, kk1 = k 32..63) with
// ONE barrier between them:
//   kk0(g): MFMAs on fragments (a0,b0) of g; ds_read the kk1 fragments of g.
//   wait lgkm; wait the LDS-DMA of step g+1 (vmcnt); s_barrier.
//   kk1(g): MFMAs on (a1,b1); ds_read the kk0 fragments of g+1 (other buffer,
//           landed: every wave passed its vmcnt before the barrier) and issue
//           the LDS-DMA pieces of step g+2 into g's buffer (free: every wave
//           holds g's fragments in registers before the barrier).
// No fragment-read latency is exposed after a barrier and each DMA has a whole
// K-step to land.  With >= 32 MFMAs per phase the DMA pieces are spread between
// MFMA groups; tiles with 16 per phase issue them up front so the other
// block's MFMAs cover the issue cost.  The DMA cursor
// runs on across the tiles of the persistent schedule.
//
// Output layout: the W (MFMA "A") fragment of column block ni, row i reads W
// row  wn + (i>>2)*4*NI + ni*4 + (i&3)  so lane (fr, fq) owns the 4*NI
// CONSECUTIVE output columns wn + fq*4*NI .. +4*NI-1 of row fr: 16-byte
// epilogue stores (half the store instructions of the 8-byte form; the
// epilogue tail is store-issue-bound).  The W LDS image is XOR-swizzled by
// sw(r) = (r & 2) | (bit (2 + log2 NI) of r) << 2, conflict-free for these
// reads and independent of ni, so every fragment offset is an immediate.
//
// Configs: 160x128 (4 waves of 80x64, or 8 of 80x32), 256x128 (8 waves,
// 4x2 of 64x64), 256x256 (8 waves, 128x64), 192x256, 224x192.  (A 4-wave 256x256 with 128x128 per wave
// needs 256 accumulator AGPRs plus > 256 VGPRs and spills: not built.)
// ---------------------------------------------------------------------------
// NS: LDS stages.  2 = the schedule above.  3 (K-long GEMMs that fit in one round of blocks,
// launch_pipe): phase1 of step g issues the DMA of step g+3 into g's buffer, and the wait
// before the barrier lets the DMA of step g+2 stay in flight, so each DMA has two K-steps to
// land instead of one (c_proj at K = 3072 with one block per CU was bound by that latency).
// LDS-DMA pieces: a K-step stages BN / 8 W pieces then BM / 8 A pieces of 1 KiB (8 rows x 64 k);
// piece q goes to wave q % NW, so a wave issues NP = ceil(pieces / NW) of them (one fewer on some
// waves when NW does not divide the count: uneven tiles, 2-stage schedule only).
// OCC: blocks per CU the tile is built for; 8-wave tiles at OCC 2 run 4 waves per SIMD (<= 128 VGPRs).
template <int NW, int OCC>
struct PipeBounds {
  static constexpr int waves_per_eu = NW == 8 && OCC >= 2 ? 4 : 2;
};

// HM = 1 (half-tile last round; 2 x 4 waves, 2-stage, no split-K): each XCD's tiles run in the plain
// strided order for F = cnt / nbx whole rounds, and the R = cnt % nbx tiles of the partial last
// round as 2R half tiles (rows m0 .. m0 + BM/2 - 1 and m0 + BM/2 .. m0 + BM - 1, full K) on 2R of the
// XCD's blocks.  On a half tile every wave takes half its rows (wave tile TM/2 x TN, MI/2 MFMA row
// groups), so both waves of each SIMD keep computing.  The last round then takes about half a
// tile's time instead of a tile's (c_fc at 12800 rows on 256x256: 75 tiles per XCD over 32 blocks,
// 2 + 11 / 32 rounds of work paid as 3 before).  No K split: every output is the same MFMA chain
// as in the whole tile.
template <typename T, int BM, int BN, int WGM, int WGN, int EPI, int ACT, int NS = 2, int OCC = 2, int RS = 0,
          int HM = 0>
__global__ __launch_bounds__(WGM* WGN * 64, (PipeBounds<WGM * WGN, OCC>::waves_per_eu)) void gemm_pipe_kernel(
    GemmParams p) {
  typedef typename Vec8<T>::type V8;
  constexpr bool LNF = epi_lnf(EPI);
  static_assert(!LNF || std::is_same<T, _Float16>::value, "LayerNorm fold: f16 operands");
  typedef typename std::conditional<EPI == EPI_LNF_BF, __bf16, T>::type OT;  // 16-bit output type
  // LDS beyond the stages: bias slots; EPI_LNF: + column-sum slots + the tile's row statistics (2 x SROWP)
  constexpr int SROWP = LNF ? (BM * 8 + 1023) / 1024 * 1024 : 0;
  constexpr int EXTRA = LNF ? 4096 + 2 * SROWP : 2048;
  constexpr int NW = WGM * WGN;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int PW = BN / 8, PA = BM / 8, PT = PW + PA;
  constexpr int NP = (PT + NW - 1) / NW;    // DMA pieces per wave and K-step
  constexpr bool EVEN = PT % NW == 0;       // every wave issues NP pieces (else waves < PT % NW issue NP, the rest NP - 1)
  constexpr bool WSPLIT = PW % NW == 0;     // piece i of every wave is a W piece iff i < PW / NW
  constexpr int TM = BM / WGM, TN = BN / WGN, MI = TM / 16, NI = TN / 16;
  constexpr int LG = NI == 2 ? 1 : NI == 4 ? 2 : 3;  // (swW: NI in {2, 4, 8})
  constexpr int NG = MI;  // MFMA groups per phase: 16 rows x all NI column blocks each
  // DMA pieces spread between MFMA groups of phase 1 (>= 32 MFMAs per phase; with
  // CLIPGPU_GEMM_SPREAD_W8, also the one-block-per-CU 8-wave tiles, whose pieces otherwise go out in
  // one burst after the step barrier while no MFMA issues), else issued up front
  constexpr bool SPREAD = MI * NI >= 32 || (CLIPGPU_GEMM_SPREAD_W8 && NW == 8 && OCC < 2) || CLIPGPU_GEMM_SPREAD_ALL;
  (void)LG;
  static_assert(BM % 8 == 0 && BN % 8 == 0 && MI >= 1 && BN <= 256 && PT >= NW, "bad tile");
  static_assert(NI == 2 || NI == 3 || NI == 4 || NI == 6 || NI == 8, "column permutation: NI in {2,3,4,6,8}");
  static_assert(NS == 2 || NS == 3, "2 or 3 LDS stages");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE + EXTRA];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // The DMA row strides, fetched with the other kernel arguments up front.  Read lazily inside
  // set_tile's per-piece (wave-dependent) branches, each became its own kernel-argument round trip:
  // five serialized s_load + s_waitcnt in the prologue (round-3 stamps; ~0.25 us per round trip,
  // tools/dispatch_probe.hip).
  const int lda_i = (int)p.lda, ldw_i = (int)p.ldw, nb = gridDim.x;
  const char* const Ab = (const char*)p.A;
  const char* const Wb = (const char*)p.W;
  const float* const bias_p = p.bias;
  const float* const cs_p = p.cs;        // EPI_LNF
  const float* const rs_p = p.rowstats;  // EPI_LNF
  asm volatile("" ::"s"(lda_i), "s"(ldw_i), "s"(nb), "s"(Ab), "s"(Wb), "s"(bias_p));
  if constexpr (LNF) asm volatile("" ::"s"(cs_p), "s"(rs_p));
  const int nTn = (p.N + BN - 1) / BN;
  const int grp = p.group > 0 ? p.group : CLIPGPU_TILE_GROUP;
  asm volatile("" ::"s"(grp));
  const int nTm = (p.M + BM - 1) / BM;
  const int ntiles = nTn * nTm;
  const int nk = p.K / BK;  // K-steps per tile

  static_assert(!HM || (NS == 2 && WGM == 2), "half tiles: 2 x N waves, 2-stage schedule");
  int t_first, t_stride, t_end;
  int hm_F = 0, hm_start = 0, hm_nbx = 1, hm_j = 0;  // HM: whole rounds, XCD range start, blocks, index
  if constexpr (HM) {
    const int x = blockIdx.x & 7, nbx = nb >> 3, j = blockIdx.x >> 3;
    const int q = ntiles >> 3, r = ntiles & 7;
    hm_start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    const int cnt = q + (x < r ? 1 : 0);
    hm_F = cnt / nbx;
    hm_nbx = nbx;
    hm_j = j;
    // units: the F whole tiles, then (blocks j < 2R) one half tile
    t_first = 0;
    t_stride = 1;
    t_end = hm_F + (j < 2 * (cnt % nbx) ? 1 : 0);
  } else if (nb % 8 == 0 && nb < ntiles) {
    const int x = blockIdx.x & 7, nbx = nb >> 3;
    const int q = ntiles >> 3, r = ntiles & 7;
    const int start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    t_first = start + (blockIdx.x >> 3);
    t_stride = nbx;
    t_end = start + q + (x < r ? 1 : 0);
  } else {
    t_first = xcd_remap(blockIdx.x, nb);
    t_stride = ntiles;
    t_end = t_first + 1;
  }
  if (t_first >= t_end) return;
  const int total = ((t_end - t_first + t_stride - 1) / t_stride) * nk;  // this block's K-steps
  auto unit_coords = [&](int u, int& m0, int& n0) {
    if constexpr (HM) {  // u < F: whole tile j + u nbx; u == F: half (j & 1) of tile F nbx + j / 2
      if (u < hm_F) {
        tile_coords(hm_start + hm_j + u * hm_nbx, nTm, nTn, BM, BN, m0, n0, grp);
      } else {
        tile_coords(hm_start + hm_F * hm_nbx + (hm_j >> 1), nTm, nTn, BM, BN, m0, n0, grp);
        m0 += (hm_j & 1) * (BM / 2);
      }
      return;
    }
    tile_coords(u, nTm, nTn, BM, BN, m0, n0, grp);
  };

  // W image swizzle for the permuted W-row reads (rowB below)
  // The swizzle must be the same for the NI rows a lane reads (rowB + 4 ni, read at immediate
  // offsets).  NI = 3 / 6: lane (fr, fq) reads rows 4 NI j + i + 4 ni of its wave's 16 NI (j = fr >> 2,
  // i = fr & 3), so swW = c(j) ^ (2 j + (i >> 1)) with c(j) = 1 for j in {1, 2} (the lanes of one
  // ds_read_b128 group pair fq with j that way) gives every group 16 distinct 16-byte slots
  // (tools/lds_swizzle_check.py checks every wave, column block and k half).
  auto swW = [](int r) {
    if constexpr (NI == 3 || NI == 6) {
      const int j = (r % (16 * NI)) / (4 * NI);
      return ((j == 1 || j == 2) ? 1 : 0) ^ (2 * j + ((r & 3) >> 1));
    } else {
      return (r & 2) | (((r >> (2 + LG)) & 1) << 2);
    }
  };

  // ---- LDS-DMA cursor (global step d_g = tile d_ti, K-step d_kt) -----------
  // poff[i]: per-lane source byte offset of this wave's piece i (q = wave + NW * i) from the
  // kernel-argument base pointer (A or W), for the current unit's first K-step.
  uint32_t poff[NP];
  auto piece_is_w = [&](int i, int q) { return WSPLIT ? (i < PW / NW) : (q < PW); };
  auto set_tile = [&](int m0, int n0) {
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int q = wave + NW * i;
      if (!EVEN && q >= PT) {
        poff[i] = 0;
      } else if (piece_is_w(i, q)) {
        const int r = q * 8 + (lane >> 3);
        const int c = (lane & 7) ^ swW(r);
        poff[i] = (uint32_t)(min(n0 + r, p.N - 1) * ldw_i + c * 8) * 2u;
      } else {
        const int r = (q - PW) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        poff[i] = (uint32_t)(min(m0 + r, p.M - 1) * lda_i + c * 8) * 2u;
      }
    }
  };
  int d_g = 0, d_kt = 0, d_t = t_first, d_n0 = 0, d_m0 = 0, d_ti = 0;
  {
    int m0, n0;
    unit_coords(d_t, m0, n0);
    set_tile(m0, n0);
    d_n0 = n0;
    d_m0 = m0;
  }
  // A piece's issue is branch-free scalar work the compiler shares across the step's pieces: the stage
  // base (d_stage, rotated instead of d_g % NS), the K-step's source bases, a wave-uniform per-piece
  // LDS offset.  Only piece NP - 1 can fall past the PT pieces (uneven splits: waves >= PT % NW skip
  // it).  (Round 6: the per-piece branches and modulos cost ~15 scalar instructions a piece, ~105 per
  // K-step and wave on the 224x192 tile -- as many issue slots as its 42 MFMAs.)
  const bool last_piece = EVEN || wave < PT % NW;
  int d_stage = 0;  // d_g % NS
  auto dma_piece = [&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if constexpr (!EVEN && i == NP - 1) {
      if (!last_piece) return;
    }
#ifdef CLIPGPU_GEMM_STAMPS
    if (p.diag & 4) return;  // timing experiment: no operand DMA in the loop (stale LDS tiles)
#endif
    const int q = wave + NW * i;
    const bool w = piece_is_w(i, q);
    char* const dst = smem + d_stage * STAGE + (w ? A_BYTES + q * 1024 : (q - PW) * 1024);
    const char* const src = (w ? Wb : Ab) + (size_t)d_kt * (BK * 2);
    GEMM_POISON(dst);
    glds16(src + poff[i], dst);
  };
  auto dma_bias = [&]() {  // the tile's bias slice, with its first K-step (tile-parity buffer)
    if (bias_p != nullptr && wave == 0 && d_kt == 0) {
      const int n = min(d_n0 + lane * 4, ((p.N - 1) / 4) * 4);
      GEMM_POISON(smem + NS * STAGE + (d_ti & 1) * 1024);
      glds16(bias_p + n, smem + NS * STAGE + (d_ti & 1) * 1024);
      if constexpr (LNF) {  // its column sums and row statistics (before the step's pieces, like the bias)
        GEMM_POISON(smem + NS * STAGE + 2048 + (d_ti & 1) * 1024);
        glds16(cs_p + n, smem + NS * STAGE + 2048 + (d_ti & 1) * 1024);
        char* const sst = smem + NS * STAGE + 4096 + (d_ti & 1) * SROWP;
#pragma unroll
        for (int i = 0; i < SROWP / 1024; ++i) {
          GEMM_POISON(sst + i * 1024);
          glds16(rs_p + (size_t)d_m0 * 2 + i * 256 + lane * 4, sst + i * 1024);
        }
      }
    }
  };
  auto dma_advance = [&]() {
    ++d_g;
    if (++d_stage == NS) d_stage = 0;
    if (++d_kt == nk) {
      d_kt = 0;
      d_t += t_stride;
      ++d_ti;
      if (d_t < t_end) {
        int m0, n0;
        unit_coords(d_t, m0, n0);
        set_tile(m0, n0);
        d_n0 = n0;
        d_m0 = m0;
      }
    }
  };
  auto dma_step = [&]() {
    if (d_g < total) {
      static_for<NP>([&](auto j) { dma_piece(j); });
      dma_bias();
    }
    dma_advance();
  };

  // ---- fragments -------------------------------------------------------------
  const int wm = (wave / WGN) * TM, wn = (wave % WGN) * TN;
  const int fr = lane & 15, fq = lane >> 4;
  // offA / offB [kk]: base of the phase-kk fragment reads.  Lane (fr, fq) reads row fr, k chunk
  // 4 kk + fq; the W rows are permuted (rowB, + 4 ni) so that a lane owns 4 NI consecutive output
  // columns.
  uint32_t offA[2], offB[2];
  {
    const int rowB = wn + (fr >> 2) * (4 * NI) + (fr & 3);  // + 4*ni
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      offA[kk] = (uint32_t)((wm + fr) * 128 + (((kk * 4 + fq) ^ (fr >> 1)) << 4));
      offB[kk] = (uint32_t)(A_BYTES + rowB * 128 + (((kk * 4 + fq) ^ swW(rowB)) << 4));
    }
  }
  // the current unit's row layout (HM half tiles: row offset (wave / WGN) * TM / 2, MI / 2 groups)
  int wm_cur = wm, mi_lim = MI;
  uint32_t offA_cur[2] = {offA[0], offA[1]};
  auto set_layout = [&](int u) {
    if constexpr (HM) {
      const bool half = u >= hm_F;
      wm_cur = half ? (wave / WGN) * (TM / 2) : wm;
      mi_lim = half ? MI / 2 : MI;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) offA_cur[kk] = offA[kk] - (uint32_t)((wm - wm_cur) * 128);
    }
    (void)u;
  };
  const uint32_t lds0 = lds_addr(smem);
  f32x4 acc[NI][MI];
  V8 a0[MI], b0[NI], a1[MI], b1[NI];  // fragments of one phase

  auto rd_b = [&](auto kc, V8(&b)[NI], uint32_t buf, int kk) {
    constexpr int k = decltype(kc)::value;
    ds_read_b128<k * 512>(b[k], buf + offB[kk]);
  };
  auto rd_a = [&](auto kc, V8(&a)[MI], uint32_t buf, int kk) {
    constexpr int k = decltype(kc)::value;
    ds_read_b128<k * 2048>(a[k], buf + offA_cur[kk]);
  };
  auto read_b = [&](V8(&b)[NI], uint32_t buf, int kk) { static_for<NI>([&](auto k) { rd_b(k, b, buf, kk); }); };
  auto read_a = [&](V8(&a)[MI], uint32_t buf, int kk) { static_for<MI>([&](auto k) { rd_a(k, a, buf, kk); }); };
  // RS = 1 (read schedule): a phase's NI + MI fragment reads for the next phase go out after the
  // first RG = NG - 2 MFMA groups, RPG per group, instead of NI up front and one A read after every
  // group, so the last read has two MFMA groups to land before the phase-end lgkmcnt wait.
  constexpr int NR = NI + MI, RG = RS ? (NG > 2 ? NG - 2 : 1) : NG, RPG = (NR + RG - 1) / RG;
  auto read_k = [&](auto kc, V8(&a)[MI], V8(&b)[NI], uint32_t buf, int kk) {
    constexpr int k = decltype(kc)::value;
    if constexpr (k < NI) rd_b(kc, b, buf, kk);
    else rd_a(std::integral_constant<int, k - NI>{}, a, buf, kk);
  };
  auto reads_after_group = [&](auto gc, V8(&a)[MI], V8(&b)[NI], uint32_t buf, int kk) {
    static_for<RPG>([&](auto j) {
      constexpr int k = (int)decltype(gc)::value * RPG + (int)decltype(j)::value;
      if constexpr ((int)decltype(gc)::value < RG && k < NR) read_k(std::integral_constant<int, k>{}, a, b, buf, kk);
    });
  };
  // MFMA group g of a phase: 16 rows x all NI column blocks; zero: the unit's first MFMA of each
  // accumulator
  auto mfma_group = [&](auto gc, V8(&a)[MI], V8(&b)[NI], auto zero) {
    constexpr int g = decltype(gc)::value;
    constexpr bool Z = decltype(zero)::value;
    if (!HM || g < mi_lim) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        acc[ni][g] = mfma_16x16x32(b[ni], a[g], Z ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[ni][g]);
    }
  };
  auto phase0 = [&](auto zero, uint32_t buf) {
    if constexpr (!RS) read_b(b1, buf, 1);
    static_for<NG>([&](auto g) {
      mfma_group(g, a0, b0, zero);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (RS) {
        reads_after_group(g, a1, b1, buf, 1);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        rd_a(g, a1, buf, 1);
      }
    });
    lgkm_wait_all(a1, b1);
  };
  auto phase1 = [&](bool next, uint32_t nbuf) {
    const bool dma = d_g < total;
    // the next step's kk0 fragments are read unconditionally (on a tile's last step from
    // the other buffer, unused): a conditional read made the compiler keep a second copy
    // of the fragment registers across the branch
    (void)next;
    if constexpr (!RS) read_b(b0, nbuf, 0);
    if (dma) {
      dma_bias();
      if constexpr (!SPREAD) static_for<NP>([&](auto j) { dma_piece(j); });
    }
    static_for<NG>([&](auto g) {
      mfma_group(g, a1, b1, std::false_type{});
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (RS) reads_after_group(g, a0, b0, nbuf, 0);
      else rd_a(g, a0, nbuf, 0);
      if constexpr (SPREAD) {
        static_for<NP>([&](auto j) {
          if constexpr (((int)j * NG) / NP == (int)g) {
            if (dma) dma_piece(j);
          }
        });
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    dma_advance();
    lgkm_wait_all(a0, b0);
  };

  // ---- epilogue: lane owns row wm+mi*16+fr, columns nc .. nc+4*NI-1 ------------
  // XE: the residual stream's element type (EPI_RESID16 / EPI_PATCH16: f16, else f32)
  auto epilogue = [&](int m0, int n0, int bpar) {
    typedef typename std::conditional<epi_x16(EPI), _Float16, float>::type XE;
    const int nc = n0 + wn + fq * (4 * NI);
    const bool nfull = nc + 4 * NI <= p.N;
    f32x4 bias[NI], csv[NI];
    // EPI_LNF: (mean, rstd) of the lane's rows, read up front -- or, on the 256-row tiles (whose
    // epilogue would spill with them), per row block inside the loop below
    constexpr bool RST_ALL = MI * NI < 32;
    f32x2 rst[RST_ALL ? MI : 1];
    const uint32_t rst_a = lds0 + NS * STAGE + 4096 + bpar * SROWP + (wm_cur + fr) * 8;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) bias[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (bias_p != nullptr) {
      const uint32_t ba = lds0 + NS * STAGE + bpar * 1024 + (wn + fq * (4 * NI)) * 4;
      static_for<NI>([&](auto ni) { ds_read_b128<(int)ni * 16>(bias[ni], ba); });
      if constexpr (LNF) {
        static_for<NI>([&](auto ni) { ds_read_b128<2048 + (int)ni * 16>(csv[ni], ba); });
        if constexpr (RST_ALL) static_for<MI>([&](auto mi) { ds_read_b64<(int)mi * 128>(rst[mi], rst_a); });
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) asm volatile("" : "+v"(bias[ni]));
      if constexpr (LNF) {
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) asm volatile("" : "+v"(csv[ni]));
        if constexpr (RST_ALL) {
#pragma unroll
          for (int mi = 0; mi < MI; ++mi) asm volatile("" : "+v"(rst[mi]));
        }
      }
    }
    // EPI_RESID adds the residual row x[m]; EPI_PATCH writes patch p of image b to token
    // row b*(G2+cls) + cls + p and adds pos[cls + p].
    constexpr bool ADDX = epi_resid(EPI) || epi_patch(EPI);
    const int G2 = p.G * p.G;
    auto out_row = [&](int m) -> long {
      if constexpr (epi_patch(EPI)) {
        const int b = m / G2;
        return ((long)b * (G2 + p.cls) + p.cls + (m - b * G2)) * p.ldo;
      } else {
        return (long)m * p.ldo;
      }
    };
    // the rows added in: the positional embedding (f32) for EPI_PATCH, the residual row (XE) for EPI_RESID
    auto add_src = [&](int m) {
      if constexpr (epi_patch(EPI)) return p.pos + (long)(p.cls + m % G2) * p.N + nc;
      else return (const XE*)p.out + (long)m * p.ldo + nc;
    };
    // The rows added in (residual x / positional embedding) are loaded before the epilogue math:
    // all MI row blocks at once when they fit in the fragment registers the main loop no longer
    // needs (MI * NI <= 20: one memory round trip instead of MI dependent ones), else a ring of
    // XR row blocks loaded XR - 1 ahead.  8-wave tiles have less register room (160x256 at 2 waves
    // per SIMD spilled with all 20 blocks up front; the 4-waves-per-SIMD builds have 128
    // registers): a ring of 3 at 2 waves per SIMD, of 2 at 4.
    constexpr bool XALL = MI * NI <= (NW == 8 ? (OCC >= 2 ? 4 : 12) : 20);
    constexpr int XRING = (NW == 8 && OCC < 2 && MI * NI <= 24) ? 3 : 2;
    constexpr int XR = XALL ? MI : (XRING < MI ? XRING : MI);
    // (the f16 residual rows stay f16 in the ring, 2 registers per 4 columns, widened at the add)
    typedef typename std::conditional<EPI == EPI_RESID16, f16x4, float4>::type XV;
    XV xr[XR][NI];
    auto load_x = [&](int mi, XV(&dst)[NI]) {
      const int m = m0 + wm_cur + mi * 16 + fr;
      if (m < p.M && nfull && (!HM || mi < mi_lim)) {
        const auto src = add_src(m);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) dst[ni] = *(const XV*)(src + ni * 4);
      }
    };
    if constexpr (ADDX) {
      if constexpr (XALL) {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) load_x(mi, xr[mi]);
      } else {
#pragma unroll
        for (int mi = 0; mi + 1 < XR; ++mi) load_x(mi, xr[mi]);
      }
    }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      if constexpr (ADDX && !XALL) {
        if (mi + XR - 1 < MI) load_x(mi + XR - 1, xr[(mi + XR - 1) % XR]);
      }
      const int m = m0 + wm_cur + mi * 16 + fr;
      if (m >= p.M || (HM && mi >= mi_lim)) continue;
      f32x2 rs = {0.f, 0.f};
      if constexpr (LNF) {
        if constexpr (RST_ALL) {
          rs = rst[mi];
        } else {
          asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(rs) : "v"(rst_a + (uint32_t)mi * 128) : "memory");
        }
      }
      float v[NI][4];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[ni][j] = LNF ? lnf_out(acc[ni][mi][j], rs[0], rs[1], csv[ni][j], bias[ni][j])
                         : acc[ni][mi][j] + bias[ni][j];
#ifdef CLIPGPU_GEMM_STAMPS
      if (p.diag & 1) {
        float s = 0.f;
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
#pragma unroll
          for (int j = 0; j < 4; ++j) s += EPI == EPI_STORE16 ? (float)to16<T>(apply_act<ACT>(v[ni][j])) : v[ni][j];
        if (s == 12345.678f) ((float*)p.out)[0] = s;
        continue;
      }
#endif
      if constexpr (epi_st16(EPI)) {
        OT* o = (OT*)p.out + (long)m * p.ldo + nc;
        if (nfull) {
          if constexpr (NI % 2 == 0) {
#pragma unroll
            for (int h = 0; h < NI / 2; ++h) {
              typename Vec8<OT>::type w;
#pragma unroll
              for (int e = 0; e < 8; ++e) w[e] = to16<OT>(apply_act<ACT>(v[2 * h + e / 4][e % 4]));
              *(typename Vec8<OT>::type*)(o + h * 8) = w;
            }
          } else {  // odd NI: the lane's 4 NI columns start 8-byte aligned only -> 8-byte stores
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) {
              typename Vec4<OT>::type w;
#pragma unroll
              for (int j = 0; j < 4; ++j) w[j] = to16<OT>(apply_act<ACT>(v[ni][j]));
              *(typename Vec4<OT>::type*)(o + ni * 4) = w;
            }
          }
        } else {
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (nc + ni * 4 + j < p.N) o[ni * 4 + j] = to16<OT>(apply_act<ACT>(v[ni][j]));
        }
      } else {
        XE* o = (XE*)p.out + out_row(m) + nc;  // (EPI_STORE32: f32)
        if (nfull) {
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            float4 w = make_float4(v[ni][0], v[ni][1], v[ni][2], v[ni][3]);
            if constexpr (ADDX) {
              const float4 x = widen4(xr[XALL ? mi : mi % XR][ni]);
              w.x += x.x; w.y += x.y; w.z += x.z; w.w += x.w;
            }
            stx4(o + ni * 4, w);
          }
        } else {
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              if (nc + ni * 4 + j >= p.N) continue;
              float r = v[ni][j];
              if constexpr (ADDX) r += (float)add_src(m)[ni * 4 + j];
              o[ni * 4 + j] = (XE)r;
            }
        }
      }
    }
  };
  // vm ops a full tile's epilogue leaves in flight behind the DMA of the step after it (the same
  // count on both paths: MI NI / 2 16-byte stores of 16-bit values, MI NI of f32, + as many loads)
  constexpr int EPI_VM = epi_st16(EPI) ? (NI % 2 ? MI * NI : MI * NI / 2)
                                            : ((epi_resid(EPI) || epi_patch(EPI)) ? 2 * MI * NI : MI * NI);
  // 3 stages: retire all but this wave's DMA pieces of the youngest step (+ X more recent vm ops):
  // NP pieces per step on waves < PT % NW (or every wave when the split is even), else NP - 1
  auto vm_wait_step = [&](auto xc) {
    constexpr int X = decltype(xc)::value;
    if (EVEN || wave < PT % NW) vm_wait<(NP + X < 63 ? NP + X : 63)>();
    else vm_wait<(NP - 1 + X < 63 ? NP - 1 + X : 63)>();
  };

  // ---- prologue: steps 0 and 1 in flight, step 0 landed, its kk0 fragments read
  GEMM_STAMP_REAL(62);
  GEMM_STAMP_HWID();
  GEMM_STAMP(0);
  // 8-wave blocks, p.prio = 1: the younger half (waves 4-7, dispatched second) at priority 1 for the
  // whole kernel, so it stops losing every issue arbitration to its SIMD partner
  // (cdna_hip_programming.md T5, static form).  The engine sets it for the vision tower: +0.75 % on
  // the two-lane ViT-B/32 bench; the text leg loses 0.5 % with it, and a per-phase priority around
  // the MFMA groups loses 0.6 % (profiles/r04_wave_priority_ab.jsonl).  Issue order only, never the sums.
  if constexpr (NW == 8) {
    if (p.prio && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  dma_step();
  vm_wait<0>();
  __builtin_amdgcn_s_barrier();
  dma_step();
  if constexpr (NS == 3) dma_step();
  read_b(b0, lds0, 0);
  read_a(a0, lds0, 0);
  lgkm_wait_all(a0, b0);
  GEMM_STAMP(1);

  int g = 0;
  int gs = 0;  // g % NS
  bool after_full_epi = false;
  int ti = 0;
  for (int t = t_first; t < t_end; t += t_stride, ++ti) {
    int m0, n0;
    unit_coords(t, m0, n0);
    GEMM_STAMP(2 + ti * 4);
    for (int kt = 0; kt < nk; ++kt, ++g) {
      if (kt + 1 == nk) GEMM_STAMP(3 + ti * 4);
      const int gs1 = gs + 1 == NS ? 0 : gs + 1;
      const uint32_t buf = lds0 + gs * STAGE;
      if (kt == 0) phase0(std::true_type{}, buf);
      else phase0(std::false_type{}, buf);
      // the DMA of step g+1 has landed once at most the later ops are outstanding: the
      // DMA of step g+2 (3 stages, if there is such a step), then the epilogue's stores
      // and loads
      constexpr int EW = EPI_VM < 63 ? EPI_VM : 63;
      if (NS == 3 && g + 2 < total) {
        if (after_full_epi) vm_wait_step(std::integral_constant<int, EPI_VM>{});
        else vm_wait_step(std::integral_constant<int, 0>{});
      } else {
#if CLIPGPU_GEMM_POISON_SELFTEST  // (the race check's own test: drop the wait on the 2-stage path)
        (void)EW;
#else
        if (after_full_epi) vm_wait<EW>();
        else vm_wait<0>();
#endif
      }
      after_full_epi = false;
#ifdef CLIPGPU_GEMM_STAMPS
      if (!(p.diag & 8)) __builtin_amdgcn_s_barrier();  // bit 3: no step barrier (timing only)
#else
      __builtin_amdgcn_s_barrier();
#endif
      phase1(kt + 1 < nk, lds0 + gs1 * STAGE);
      gs = gs1;
      if (ti == 0 && kt + 1 < nk && 34 + kt < 61) GEMM_STAMP(34 + kt);  // (slots 61-63: HW_ID, realtime)
    }
    GEMM_STAMP(4 + ti * 4);
    // (CLIPGPU_GEMM_EPI_DMA_WAIT, default on) retire this wave's LDS-DMA of the next step(s) before
    // the epilogue's stores (3 stages: all but the youngest step's pieces), so that the counted
    // wait after a full epilogue never relies on a store retiring after an older LDS-DMA (the
    // compiler's own wait insertion treats mixed pending VMEM reads and writes as unordered).
    // DESIGN.md §3 (race check) and §10 (round 3) record what this was and was not.
#if CLIPGPU_GEMM_EPI_DMA_WAIT
    if constexpr (NS == 3) vm_wait_step(std::integral_constant<int, 0>{});
    else vm_wait<0>();
#endif
    epilogue(m0, n0, ti & 1);
    // partial tiles and half tiles issue fewer vm ops than EPI_VM: drain them
    after_full_epi = m0 + BM <= p.M && n0 + BN <= p.N && (!HM || t < hm_F);
    if (!after_full_epi) vm_wait<0>();
    if (t + t_stride < t_end) {  // the next tile's step 0 landed at the last barrier
      const uint32_t buf = lds0 + gs * STAGE;
      set_layout(t + t_stride);
      read_b(b0, buf, 0);
      read_a(a0, buf, 0);
      lgkm_wait_all(a0, b0);
    }
    GEMM_STAMP(5 + ti * 4);
  }
  GEMM_STAMP_REAL(63);
}

// Persistent grids (the launchers below and gemm_grid use these, so the bench's per-site block counts
// are the launches' own).
// OCC: resident blocks per CU the tile's registers allow (4-wave tiles: up to 3 by LDS; 8-wave
// tiles: 1, or 2 when built for 4 waves per SIMD).  2 LDS stages.
constexpr int pipe_kocc(int NW, int OCC) { return NW == 8 ? (OCC >= 2 ? 2 : 1) : 2; }  // launch bounds' OCC
inline int pipe_grid(int BM, int BN, int NW, int OCC, int M, int N) {
  const int ntiles = ((N + BN - 1) / BN) * ((M + BM - 1) / BM);
  // resident blocks per CU: by LDS (2 stages + 2 KiB bias) and by registers (OCC)
  const int lds = 2 * (BM + BN) * BK * 2 + 2048;
  const int per_cu = std::max(1, std::min(NW == 8 ? pipe_kocc(NW, OCC) : OCC, (160 * 1024) / lds));
  const int resident = device_cus() * per_cu;
  if (CLIPGPU_GEMM_NONPERSIST) return ntiles;  // (A/B build: one tile per block)
  return ntiles <= resident ? ntiles : resident;
}
// Half-tile last round for the 256x256 RS tile: applies when every XCD has >= 1 whole round and at
// most nbx / 2 remainder tiles.
inline bool half_round_applies(int M, int N) {
  const int nb = device_cus();
  const int ntiles = ((N + 255) / 256) * ((M + 255) / 256);
  bool ok = nb % 8 == 0 && ntiles % nb != 0;
  const int nbx = nb >> 3, q = ntiles >> 3, r = ntiles & 7;
  for (int x = 0; ok && x < 8; ++x) {
    const int cnt = q + (x < r ? 1 : 0);
    ok = cnt >= nbx && 2 * (cnt % nbx) <= nbx;
  }
  return ok;
}
inline int grid_224(int M, int N) { return std::min(((N + 191) / 192) * ((M + 223) / 224), device_cus()); }

template <typename T, int BM, int BN, int WGM, int WGN, int EPI, int ACT, int OCC = 3, int RS = 0>
hipError_t launch_pipe(const GemmParams& p, hipStream_t s) {
  constexpr int NW = WGM * WGN;
  constexpr int KOCC = pipe_kocc(NW, OCC);
  const int grid = pipe_grid(BM, BN, NW, OCC, p.M, p.N);
  gemm_launch(gemm_pipe_kernel<T, BM, BN, WGM, WGN, EPI, ACT, 2, KOCC, RS, 0>, grid, NW * 64, s, p);
  return hipGetLastError();
}

// Half-tile last round for the 256x256 RS tile (gemm_pipe_kernel HM = 1, one block per CU): when the
// tiles leave a partial last round of at most nbx / 2 tiles per XCD after >= 1 whole round; else the
// plain RS launch (the same sums, bit for bit).
template <typename T, int EPI, int ACT>
hipError_t launch_pipe_half(const GemmParams& p, hipStream_t s) {
  if (!half_round_applies(p.M, p.N)) return launch_pipe<T, 256, 256, 2, 4, EPI, ACT, 3, 1>(p, s);
  gemm_launch(gemm_pipe_kernel<T, 256, 256, 2, 4, EPI, ACT, 2, 2, 1, 1>, device_cus(), 512, s, p);
  return hipGetLastError();
}

// 224x192, 8 waves (2 x 4 of 112 x 48), one block per CU, 3 LDS stages (156 KiB + the bias slots) when
// every tile has >= 3 K-steps: the N = width residual GEMMs of ViT-B/32 at 12800 rows are 58 x 4 = 232
// tiles, one round on 232 CUs, at 103 FLOP per staged byte (the 2-blocks-per-CU 160 x 128 tiles: 71) and
// two K-steps of LDS-DMA in flight per CU (106 KiB; 160 x 128 pairs: 72 KiB).
template <typename T, int EPI, int ACT>
hipError_t launch_pipe_224(const GemmParams& p, hipStream_t s) {
  const int grid = grid_224(p.M, p.N);
  if (p.K / BK >= 3) gemm_launch(gemm_pipe_kernel<T, 224, 192, 2, 4, EPI, ACT, 3, 1, 1, 0>, grid, 512, s, p);
  else gemm_launch(gemm_pipe_kernel<T, 224, 192, 2, 4, EPI, ACT, 2, 1, 1, 0>, grid, 512, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Skinny GEMM (M <= SKINNY_MAX_M; the pruned last layer at M = batch, the heads' projections).
// A 128-row tile there leaves most CUs idle and runs K/64 dependent K-steps, each paying an
// L2/HBM round trip (c_proj at M = 128: 6 tiles, 48 steps, 53 us).  Instead one wave owns one
// 16x16 output block and streams its W rows and A rows straight from global memory (both
// L2-resident at these sizes), two batches of U = 8 k-chunks of loads in flight ahead of the MFMAs.
// Operand roles, the k -> lane assignment (lane (fr, fq) holds k = 32c + 8fq .. +7 of row fr)
// and the K order of the MFMA chain are those of the tiled kernels, and the epilogue does the
// same float ops, so every output element is bit-identical to theirs
// (test_skinny_gemm_is_bit_exact, test_last_layer_pruning_is_bit_exact).
//
// GEN = 1 (U = 2) is the general form for the shapes the pipelined kernel does not take -- K = 64
// (one K-step), 16-bit outputs whose row pitch is not a multiple of 8 elements -- at any M, with N
// tails (clamped W rows, masked stores) and element stores where a row is not 4-aligned.  Round 6
// removed the 128x128 "bt" kernel that used to take these shapes: its run-to-run wrong outputs
// (one accumulator register of one lane quarter) were never root-caused, and this
// form gives the pipelined tiles' bits by construction (test_general_gemm_is_bit_exact).
constexpr int SKINNY_MAX_M = 256;
constexpr int SKINNY_U = 8;

template <typename T, int EPI, int ACT, int U = SKINNY_U, int GEN = 0>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(GemmParams p) {
  typedef typename Vec8<T>::type V8;
  constexpr bool LNF = epi_lnf(EPI);
  static_assert(!LNF || std::is_same<T, _Float16>::value, "LayerNorm fold: f16 operands");
  static_assert(!epi_patch(EPI), "the patch GEMM always has K >= 128 (pipelined tiles)");
  typedef typename std::conditional<EPI == EPI_LNF_BF, __bf16, T>::type OT;  // 16-bit output type
  const int lane = threadIdx.x & 63;
  const long wid = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nTn = GEN ? (p.N + 15) >> 4 : p.N >> 4;
  const long tm = wid / nTn;
  const int tn = (int)(wid - tm * nTn);  // a block's 4 waves share the A rows
  if (tm * 16 >= p.M) return;
  const int fr = lane & 15, fq = lane >> 4;
  const int m = (int)tm * 16 + fr;
  const T* a = (const T*)p.A + (long)min(m, p.M - 1) * p.lda + fq * 8;
  const T* w = (const T*)p.W + (long)(GEN ? min(tn * 16 + fr, p.N - 1) : tn * 16 + fr) * p.ldw + fq * 8;
  const int nc = p.K >> 5;
  // three register batches of U k-chunks: the loads of batch i+2 are issued before the
  // MFMAs of batch i, so two batches of L2 / HBM latency are covered
  V8 w0[U], a0[U], w1[U], a1[U], w2[U], a2[U];
  auto load = [&](V8(&wv)[U], V8(&av)[U], int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      wv[u] = *(const V8*)(w + (c + u) * 32);
      av[u] = *(const V8*)(a + (c + u) * 32);
    }
  };
  load(w0, a0, 0);
  if (U < nc) load(w1, a1, U);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < nc; c0 += U) {
    if (c0 + 2 * U < nc) load(w2, a2, c0 + 2 * U);
#pragma unroll
    for (int u = 0; u < U; ++u) acc = mfma_16x16x32(w0[u], a0[u], acc);

#pragma unroll
    for (int u = 0; u < U; ++u) {
      w0[u] = w1[u];
      a0[u] = a1[u];
      w1[u] = w2[u];
      a1[u] = a2[u];
    }
  }
  if (m >= p.M) return;
  const int n = tn * 16 + fq * 4;
  if (GEN && n >= p.N) return;
  // GEN: whole, 4-aligned column groups take the vector loads / stores below (N % 4 == 0 and
  // ldo % 4 == 0); the rest go element by element
  const bool vec = !GEN || (n + 4 <= p.N && p.ldo % 4 == 0);
  f32x4 bias = {0.f, 0.f, 0.f, 0.f}, csv = {0.f, 0.f, 0.f, 0.f};
  f32x2 rst = {0.f, 0.f};
  if (p.bias != nullptr) {
    if (!GEN || n + 4 <= p.N) bias = *(const f32x4*)(p.bias + n);
    else
      for (int j = 0; j < 4; ++j) bias[j] = n + j < p.N ? p.bias[n + j] : 0.f;
  }
  if constexpr (LNF) {
    if (!GEN || n + 4 <= p.N) csv = *(const f32x4*)(p.cs + n);
    else
      for (int j = 0; j < 4; ++j) csv[j] = n + j < p.N ? p.cs[n + j] : 0.f;
    rst = *(const f32x2*)(p.rowstats + (long)m * 2);
  }
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = LNF ? lnf_out(acc[j], rst[0], rst[1], csv[j], bias[j]) : acc[j] + bias[j];
  if constexpr (epi_st16(EPI)) {
    OT* o = (OT*)p.out + (long)m * p.ldo + n;
    if (vec) {
      typename Vec4<OT>::type ov;
#pragma unroll
      for (int j = 0; j < 4; ++j) ov[j] = to16<OT>(apply_act<ACT>(v[j]));
      *(typename Vec4<OT>::type*)o = ov;
    } else {
      for (int j = 0; j < 4; ++j)
        if (n + j < p.N) o[j] = to16<OT>(apply_act<ACT>(v[j]));
    }
  } else {
    typedef typename std::conditional<epi_x16(EPI), _Float16, float>::type XE;  // (EPI_STORE32: f32)
    XE* o = (XE*)p.out + (long)m * p.ldo + n;
    if (vec) {
      float4 r = make_float4(v[0], v[1], v[2], v[3]);
      if constexpr (epi_resid(EPI)) {
        const float4 x = ldx4(o);
        r.x += x.x; r.y += x.y; r.z += x.z; r.w += x.w;
      }
      stx4(o, r);
    } else {
      for (int j = 0; j < 4; ++j) {
        if (n + j >= p.N) continue;
        float r = v[j];
        if constexpr (epi_resid(EPI)) r += (float)o[j];
        o[j] = (XE)r;
      }
    }
  }
}

// Shapes the skinny kernel takes: A_ROWS operands, 16-aligned N, K a multiple of 32*U,
// 16-byte aligned rows, no split-K.
inline bool skinny_ok(const GemmParams& p) {
  return p.M > 0 && p.M <= SKINNY_MAX_M && p.N % 16 == 0 && p.K % (32 * SKINNY_U) == 0 && p.lda % 8 == 0 &&
         p.ldw % 8 == 0 && p.ldo % 4 == 0;
}
// The general form: K % 64 == 0 (launch_gemm checks), 16-byte aligned operand rows.
inline bool general_ok(const GemmParams& p) { return p.lda % 8 == 0 && p.ldw % 8 == 0; }
inline long skinny_waves(int M, int N) { return (long)((M + 15) / 16) * ((N + 15) / 16); }

template <typename T, int EPI, int ACT, int U = SKINNY_U, int GEN = 0>
hipError_t launch_skinny(const GemmParams& p, hipStream_t s) {
  const long blocks = (skinny_waves(p.M, p.N) + 3) / 4;
  if (blocks > 0x7fffffffL) return hipErrorInvalidValue;
  gemm_launch(gemm_skinny_kernel<T, EPI, ACT, U, GEN>, (int)blocks, 256, s, p);
  return hipGetLastError();
}

template <typename T, int EPI, int ACT>
hipError_t launch_tile(const GemmParams& p, hipStream_t s) {
  if constexpr (!epi_patch(EPI)) {
    if ((p.tile == TILE_AUTO || p.tile == TILE_SKINNY) && skinny_ok(p)) return launch_skinny<T, EPI, ACT>(p, s);
  }
  if (p.tile == TILE_SKINNY) return hipErrorInvalidValue;
  const int tile = p.tile == TILE_AUTO ? pick_gemm_tile(p.M, p.N, p.K) : p.tile;
  if (tile != TILE_GENERAL && !gemm_tile_built(tile)) return hipErrorInvalidValue;
  // software-pipelined kernel: K >= 128, 16-byte-aligned 16-bit output rows
  const bool pipe = tile != TILE_GENERAL && p.K >= 2 * BK && (!epi_st16(EPI) || p.ldo % 8 == 0);
  if (!pipe) {
    // the general one-wave-per-16x16 form (any M; K = 64, unaligned 16-bit rows): the same bits
    if constexpr (epi_patch(EPI)) {
      return hipErrorInvalidValue;
    } else {
      if (!general_ok(p)) return hipErrorInvalidValue;
      return launch_skinny<T, EPI, ACT, 2, 1>(p, s);
    }
  }
  if constexpr (epi_lnf(EPI)) {
    // EPI_LNF: the 224x192 tile's three stages leave no LDS for the row statistics; it runs the
    // 4-wave 160x128 RS tile instead (the same bits: every tile computes the same sums)
    switch (tile) {
      case TILE_256x128: return launch_pipe<T, 256, 128, 4, 2, EPI, ACT>(p, s);
      case TILE_256x256: return launch_pipe<T, 256, 256, 2, 4, EPI, ACT>(p, s);
      case TILE_192x256_W8: return launch_pipe<T, 192, 256, 2, 4, EPI, ACT, 1>(p, s);
      case TILE_256x256_RS: return launch_pipe<T, 256, 256, 2, 4, EPI, ACT, 3, 1>(p, s);
      case TILE_160x128_RS: return launch_pipe<T, 160, 128, 2, 2, EPI, ACT, 3, 1>(p, s);
      case TILE_160x128_W8_RS: return launch_pipe<T, 160, 128, 2, 4, EPI, ACT, 2, 1>(p, s);
      case TILE_256x256_HALF: return launch_pipe_half<T, EPI, ACT>(p, s);
      case TILE_224x192_W8: return launch_pipe<T, 160, 128, 2, 2, EPI, ACT, 3, 1>(p, s);
      default: break;
    }
  } else {
    switch (tile) {
      case TILE_256x128: return launch_pipe<T, 256, 128, 4, 2, EPI, ACT>(p, s);
      case TILE_256x256: return launch_pipe<T, 256, 256, 2, 4, EPI, ACT>(p, s);
      case TILE_192x256_W8: return launch_pipe<T, 192, 256, 2, 4, EPI, ACT, 1>(p, s);
      case TILE_256x256_RS: return launch_pipe<T, 256, 256, 2, 4, EPI, ACT, 3, 1>(p, s);
      case TILE_160x128_RS: return launch_pipe<T, 160, 128, 2, 2, EPI, ACT, 3, 1>(p, s);
      case TILE_160x128_W8_RS: return launch_pipe<T, 160, 128, 2, 4, EPI, ACT, 2, 1>(p, s);
      case TILE_256x256_HALF: return launch_pipe_half<T, EPI, ACT>(p, s);
      case TILE_224x192_W8: return launch_pipe_224<T, EPI, ACT>(p, s);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

template <typename T>
hipError_t launch_typed(int epi, int act, const GemmParams& p, hipStream_t s) {
  switch (epi) {
    case EPI_STORE16:
      switch (act) {
        case ACT_NONE: return launch_tile<T, EPI_STORE16, ACT_NONE>(p, s);
        case ACT_QUICK_GELU: return launch_tile<T, EPI_STORE16, ACT_QUICK_GELU>(p, s);
        case ACT_GELU: return launch_tile<T, EPI_STORE16, ACT_GELU>(p, s);
        case ACT_GELU_TANH: return launch_tile<T, EPI_STORE16, ACT_GELU_TANH>(p, s);
      }
      break;
    case EPI_RESID:  // the residual stream: f32, or f16 (GemmParams.x16)
      return p.x16 ? launch_tile<T, EPI_RESID16, ACT_NONE>(p, s) : launch_tile<T, EPI_RESID, ACT_NONE>(p, s);
    case EPI_STORE32: return launch_tile<T, EPI_STORE32, ACT_NONE>(p, s);
    case EPI_PATCH:  // rows from launch_patch_rows
      return p.x16 ? launch_tile<T, EPI_PATCH16, ACT_NONE>(p, s) : launch_tile<T, EPI_PATCH, ACT_NONE>(p, s);
    case EPI_LNF:
    case EPI_LNF_BF:  // f16 operands only (launch_gemm); the CLIP trunk's activations
      if constexpr (std::is_same<T, _Float16>::value) {
        if (epi == EPI_LNF) {
          switch (act) {
            case ACT_NONE: return launch_tile<T, EPI_LNF, ACT_NONE>(p, s);
            case ACT_QUICK_GELU: return launch_tile<T, EPI_LNF, ACT_QUICK_GELU>(p, s);
            case ACT_GELU: return launch_tile<T, EPI_LNF, ACT_GELU>(p, s);
          }
        } else {
          switch (act) {
            case ACT_NONE: return launch_tile<T, EPI_LNF_BF, ACT_NONE>(p, s);
            case ACT_QUICK_GELU: return launch_tile<T, EPI_LNF_BF, ACT_QUICK_GELU>(p, s);
            case ACT_GELU: return launch_tile<T, EPI_LNF_BF, ACT_GELU>(p, s);
          }
        }
      }
      break;
  }
  return hipErrorInvalidValue;
}

}  // namespace

int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      cus = prop.multiProcessorCount;
    if (cus <= 0) cus = 256;
  }
  return cus;
}


// Blocks (the persistent grid) of one launch of `tile` (a GemmTile id; TILE_AUTO resolved as launch_tile
// does, the skinny kernel included) at M x N x K with row operands: the launchers' own grid functions.
int gemm_grid(int tile, int M, int N, int K) {
  GemmParams p{};
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = p.ldw = K;
  p.ldo = N;
  if ((tile == TILE_AUTO || tile == TILE_SKINNY) && skinny_ok(p)) return (int)((skinny_waves(M, N) + 3) / 4);
  if (tile == TILE_AUTO) tile = pick_gemm_tile(M, N, K);
  if (K >= 2 * BK && tile != TILE_GENERAL) {
    switch (tile) {
      case TILE_256x128: return pipe_grid(256, 128, 8, 3, M, N);
      case TILE_256x256: return pipe_grid(256, 256, 8, 3, M, N);
      case TILE_192x256_W8: return pipe_grid(192, 256, 8, 1, M, N);
      case TILE_256x256_RS: return pipe_grid(256, 256, 8, 3, M, N);
      case TILE_160x128_RS: return pipe_grid(160, 128, 4, 3, M, N);
      case TILE_160x128_W8_RS: return pipe_grid(160, 128, 8, 2, M, N);
      case TILE_256x256_HALF: return half_round_applies(M, N) ? device_cus() : pipe_grid(256, 256, 8, 3, M, N);
      case TILE_224x192_W8: return grid_224(M, N);
      default: break;
    }
  }
  return (int)std::min<long>((skinny_waves(M, N) + 3) / 4, 0x7fffffffL);  // the general form
}

// Tile choice: large-M GEMMs use the 256-row tiles (128 FLOP per staged byte
// instead of 64); among those, the column tile that wastes the least of the
// last wave of blocks over the 256 CUs (one 8-wave block per CU).
int pick_gemm_tile(int M, int N, int K) {
  // Small M: the 4-wave 160x128 pipelined tile (launch_tile sends K < 128 to the general form).
  (void)K;
  if (M < 2048) return TILE_160x128_RS;
  const int cus = 256;
  auto eff = [&](int bm, int bn) {
    const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    const long rounds = (tiles + cus - 1) / cus;
    return (double)tiles / (double)(rounds * cus);
  };
  // 256x128 stages 1.5x the bytes per FLOP of 256x256: prefer 256x256 unless it idles
  // noticeably more CUs in the tail.
  return eff(256, 256) >= 0.85 * eff(256, 128) ? TILE_256x256 : TILE_256x128;
}

// Rows one launch may cover: the kernels address their operands with 32-bit per-lane byte offsets
// from the kernel-argument base pointers (SGPR base + VGPR offset DMA), so a launch keeps
// rows * lda * 2 bytes under 2^31.  Larger M runs as consecutive row chunks (launch_gemm below);
// every output row is the same MFMA chain whichever launch computes it, so the chunking is
// bit-invisible (test_gemm_row_chunks_are_bit_exact, the SO400M max_batch 1024 test).
// Test hook (clipgpu_test_gemm_chunk_rows): a smaller row cap for the chunked path, so the tests run it
// at small batches (0 = off).
long g_gemm_chunk_cap = 0;

long gemm_chunk_rows(long lda, int G) {
  long rows = ((1L << 31) - 1) / (2 * lda);
  if (g_gemm_chunk_cap > 0) rows = std::min(rows, g_gemm_chunk_cap);
  rows -= rows % 256;                           // whole 256-row tiles
  if (G > 0) rows -= rows % ((long)G * G);      // EPI_PATCH: whole images
  return rows;
}

// EPI_LNF: f16 operands, output in dt (EPI_LNF_BF for bf16); bias and column sums required.
hipError_t launch_dt(DType dt, int epi, int act, const GemmParams& p, hipStream_t s) {
  if (epi == EPI_LNF) return launch_typed<_Float16>(dt == DT_BF16 ? EPI_LNF_BF : EPI_LNF, act, p, s);
  return dt == DT_BF16 ? launch_typed<__bf16>(epi, act, p, s) : launch_typed<_Float16>(epi, act, p, s);
}

hipError_t launch_gemm(DType dt, int asrc, int epi, int act, const GemmParams& p, hipStream_t s) {
  if (p.K % BK != 0 || p.M <= 0 || p.N <= 0) return hipErrorInvalidValue;
  if (epi == EPI_LNF && (p.bias == nullptr || p.cs == nullptr || p.rowstats == nullptr || p.N % 4 != 0))
    return hipErrorInvalidValue;
  if (epi == EPI_LNF_BF) return hipErrorInvalidValue;  // internal code
  if (p.bias != nullptr && p.N % 4 != 0) return hipErrorInvalidValue;  // 16-byte bias DMA
  // 32-bit staging offsets: W must fit whole; A is chunked by rows
  if ((long)p.N * p.ldw * 2 >= (1L << 31) || p.lda <= 0) return hipErrorInvalidValue;
  if (asrc != A_ROWS) return hipErrorInvalidValue;  // pixels go through launch_patch_rows first
  if ((long)p.M * p.lda * 2 >= (1L << 31) || (g_gemm_chunk_cap > 0 && p.M > g_gemm_chunk_cap)) {
    const int G = epi == EPI_PATCH ? p.G : 0;
    const long chunk = gemm_chunk_rows(p.lda, G);
    if (chunk <= 0) return hipErrorInvalidValue;
    // output element size: 16-bit activations, the f16 residual stream (x16), else f32
    const long osz = (epi_st16(epi) || ((epi == EPI_RESID || epi == EPI_PATCH) && p.x16)) ? 2 : 4;
    for (long m0 = 0; m0 < p.M; m0 += chunk) {
      GemmParams q = p;
      q.M = (int)std::min<long>(chunk, p.M - m0);
      q.A = (const char*)p.A + m0 * p.lda * 2;
      if (epi == EPI_LNF) q.rowstats = p.rowstats + 2 * m0;  // (mean, rstd) of the chunk's rows
      const long orow = G > 0 ? m0 / ((long)G * G) * ((long)G * G + p.cls) : m0;  // EPI_PATCH: token rows
      q.out = (char*)p.out + orow * p.ldo * osz;
      const hipError_t err = launch_dt(dt, epi, act, q, s);
      if (err != hipSuccess) return err;
    }
    return hipSuccess;
  }
  return launch_dt(dt, epi, act, p, s);
}

#ifdef CLIPGPU_GEMM_STAMPS
hipError_t read_gemm_stamps(unsigned long long* host, int nblocks, bool clear) {
  const size_t n = (size_t)std::min(nblocks, kStampBlocks) * kStampSlots * sizeof(unsigned long long);
  if (clear) {
    static unsigned long long zeros[kStampBlocks * kStampSlots];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_stamps), zeros, sizeof(zeros));
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_stamps), n);
}
#endif

}  // namespace clipgpu
