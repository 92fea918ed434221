// Host-visible launchers for the clipgpu gfx950 kernels.  All launchers are
// asynchronous on `stream` and never allocate, copy or synchronise (so a
// forward can be captured into a hipGraph).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace clipgpu {

enum DType { DT_BF16 = 0, DT_F16 = 1 };

// Source of the GEMM A operand (launch_gemm takes A_ROWS only) / of the patch rows.
enum ASrc {
  A_ROWS = 0,     // T16 [M][lda], staged by global_load_lds
  A_IMG_F32 = 1,  // launch_patch_rows: normalised f32 NCHW pixels
  A_IMG_U8 = 2,   // launch_patch_rows: u8 NHWC pixels, normalised on load
};
// GEMM epilogue.
enum Epi {
  EPI_STORE16 = 0,  // out16[m][n] = act(acc + bias[n])
  EPI_RESID = 1,    // out32[m][n] += acc + bias[n]        (residual stream, in place)
  EPI_STORE32 = 2,  // out32[m][n] = acc + bias[n]
  EPI_PATCH = 3,    // x[b*(G^2+cls) + cls + p][n] = acc + bias[n] + pos[cls + p][n]
  EPI_STOREQ = 4,   // launch_gemm_mx only: out = MX-fp8 of act(acc + bias[n]) (e4m3 + scales)
  // (internal: the residual-stream epilogues with an f16 stream, GemmParams.x16; launch_gemm picks them)
  EPI_RESID16 = 5,
  EPI_PATCH16 = 6,
  // LayerNorm folded into the GEMM (A = the f16 residual stream x itself, W' = W diag(gamma) in f16):
  //   out16[m][n] = act(rstd_m (acc - mean_m cs[n]) + bias[n]),  cs[n] = sum_k W'[n][k]
  //   (GemmParams.cs), bias = b + W beta, (mean_m, rstd_m) = GemmParams.rowstats[m] (launch_ln_stats).
  //   launch_gemm takes EPI_LNF with dt = the output type; the operands are f16.
  EPI_LNF = 7,
  EPI_LNF_BF = 8,  // (internal: EPI_LNF with a bf16 output)
};
constexpr bool epi_resid(int e) { return e == EPI_RESID || e == EPI_RESID16; }
constexpr bool epi_patch(int e) { return e == EPI_PATCH || e == EPI_PATCH16; }
constexpr bool epi_x16(int e) { return e == EPI_RESID16 || e == EPI_PATCH16; }
constexpr bool epi_lnf(int e) { return e == EPI_LNF || e == EPI_LNF_BF; }
constexpr bool epi_st16(int e) { return e == EPI_STORE16 || epi_lnf(e); }  // 16-bit activation outputs

struct GemmParams {
  const void* A; long lda;   // A_ROWS source
  const void* W; long ldw;   // [N][K] 16-bit weights
  const float* bias;         // [N] or nullptr
  void* out; long ldo;
  int M, N, K;
  int G;                     // EPI_PATCH: patch grid (G^2 patch rows per image)
  int cls;                   // EPI_PATCH: 1 = token 0 of each image is a class token (rows / pos shifted by one)
  const float* pos;          // EPI_PATCH positional embedding [G^2+cls][N]
  int tile;                  // GemmTile (0 = pick by shape)
  int diag;                  // stamp build only: bit 0 = skip epilogue stores, bit 2 = no operand DMA, bit 3 = no step barrier
  int group;                 // tile order: row panels per group (gemm_util.hpp tile_coords); 0 = 8
  int prio;                  // 8-wave gemm_pipe tiles: 1 = the younger half of the block at s_setprio 1
  int x16;                   // EPI_RESID / EPI_PATCH: the residual stream `out` is f16 (else f32); the adds are f32
  const float* cs;           // EPI_LNF: [N] column sums of W' (f32)
  const float* rowstats;     // EPI_LNF: [M + 256][2] (mean, rstd) of A's rows (rows >= M are read, unused)
};

// Tile configurations of the MFMA GEMM.  Ids are stable across rounds; the ones not listed were
// experiment tiles that never won a site (round 4 removed them from the library: DESIGN.md §10 keeps
// their measurements): 4-12 and 16 (4- / 8-wave 128-192-row variants), 19-20 (ping-pong schedule),
// 21-25 (32x32x16 MFMA), 27 (spread-DMA 224x192), 28 (224x192 at 4 waves of 112x96, one per SIMD: the
// same speed as 26, round 6).
enum GemmTile {
  TILE_AUTO = 0,
  // (1: the 128x128 "bt" kernel, removed in round 6 -- run-to-run wrong outputs; its
  // shapes, K < 128 and unaligned 16-bit rows, run the skinny kernel's general form)
  TILE_256x128 = 2,       // gemm_pipe_kernel: 8 waves (4x2, 64x64 each), 96 KiB LDS (shape heuristic)
  TILE_256x256 = 3,       // gemm_pipe_kernel: 8 waves (2x4, 128x64 each), 128 KiB LDS (shape heuristic)
  TILE_192x256_W8 = 13,   // 2x4 waves of 96x64, 114 KiB LDS, 1 block / CU (the table's ViT-H/14 c_proj)
  // the spread fragment-read schedule (gemm_pipe_kernel RS = 1: a phase's reads for the next phase go
  // out over its first MI - 2 MFMA groups); bit-identical to the others, speed only
  TILE_256x256_RS = 14,
  TILE_160x128_RS = 15,     // 4 waves of 80x64, 74 KiB LDS, 2 blocks / CU (small M; the table's vision c_fc / c_proj /
                            // patch and large-text c_proj)
  TILE_160x128_W8_RS = 17,  // 2x4 waves of 80x32, 74 KiB LDS, 2 blocks / CU (the table's N = width sites)
  TILE_256x256_HALF = 18,   // 256x256 RS with the partial last round as half tiles (HM = 1; the table's
                            // qkv / c_fc)
  // 2x4 waves of 112x48 (RS), 1 block / CU, 3 LDS stages (158 KiB) when K >= 192: the N = 768 residual
  // GEMMs at 12800 rows are 232 tiles, one round
  TILE_224x192_W8 = 26,
  TILE_SKINNY = 100,      // gemm_skinny_kernel: one wave per 16x16 block, M <= 256 (TILE_AUTO's pick there)
  TILE_GENERAL = 101,     // gemm_skinny_kernel's general form, any M / N (the pick where no pipelined tile runs)
};
// The GemmTile ids the library builds (pins, tests and the timing tuner take only these).
constexpr int kGemmTiles[] = {TILE_256x128, TILE_256x256, TILE_192x256_W8, TILE_256x256_RS,
                              TILE_160x128_RS, TILE_160x128_W8_RS, TILE_256x256_HALF, TILE_224x192_W8};
inline bool gemm_tile_built(int t) {
  for (int k : kGemmTiles)
    if (k == t) return true;
  return false;
}
int pick_gemm_tile(int M, int N, int K);
// Test hook: cap on the rows of one launch of launch_gemm's row-chunked path (0 = only the 2^31-byte
// operand limit chunks).  Chunking is bit-invisible (test_chunked_gemm_launches_are_bit_exact).
extern long g_gemm_chunk_cap;
int gemm_grid(int tile, int M, int N, int K);  // blocks of one launch (the persistent grid)
int device_cus();  // CUs of the current device (cached)

// act: Act enum from common.hpp (only used with EPI_STORE16)
hipError_t launch_gemm(DType dt, int asrc, int epi, int act, const GemmParams& p, hipStream_t s);
// Kernel-boundary timing of the next GEMM launch on this thread (clipgpu_profile_*): when
// both events are set, launch_gemm launches through hipExtLaunchKernelGGL with them, so the
// events stamp the kernel's own start and end (an event pair recorded around a launch also
// times its dispatch), then clears them.
struct GemmLaunchEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local GemmLaunchEvents g_gemm_events;

// Multi-head self-attention over packed qkv rows [B*N][3*D] -> out [B*N][D];
// head_dim must be 64; N <= 256.
// MAP attention pool (timm AttentionPoolLatent, one latent query): q [D] f32 (shared by all
// images), kv [B*N][2D] 16-bit = [k | v], out [B][D] 16-bit (heads concatenated).
hipError_t launch_map_attention(DType dt, const float* q, const void* kv, void* out, int B, int N, int H, int D,
                                hipStream_t s);
hipError_t launch_attention(DType dt, const void* qkv, void* out, int B, int N, int H, int D,
                            int causal, hipStream_t s);

// The residual stream x (launchers taking `x, x16`): f32 rows, or f16 rows when x16 != 0
// (clipgpu_options.residual); every add into it and every statistic of it is computed in f32.
// stats[r] = (mean, 1 / sqrt(var + eps)) of x[r] for r < rows, as launch_ln_rows computes them
// (the EPI_LNF GEMMs' GemmParams.rowstats).
hipError_t launch_ln_stats(const void* x, int x16, float eps, float* stats, int rows, int D, hipStream_t s);
// out16[r] = LN(x[r]) for r < rows.
hipError_t launch_ln_rows(DType dt, const void* x, int x16, const float* w, const float* b, float eps,
                          void* out16, int rows, int D, hipStream_t s, uint8_t* qs = nullptr);
// qs != nullptr (these LN launchers): the output is MX-fp8, out16 = e4m3 bytes [rows][D],
// qs = scales [rows][D/32] (gemm_mx.hip's A operand); D % 32 == 0.

// Vision stem tail: CLS row = cls + pos[0]; x = ln_pre(x) (in place); h = ln_1(x) -- or, h == nullptr,
// stats = ln_1's row statistics (launch_ln_stats; the LayerNorm-folded QKV GEMM).
hipError_t launch_vision_embed_ln(DType dt, void* x, int x16, const float* cls, const float* pos,
                                  const float* lnpre_w, const float* lnpre_b,
                                  const float* ln1_w, const float* ln1_b, float eps,
                                  void* h, int B, int tokens, int D, hipStream_t s, uint8_t* qs = nullptr,
                                  float* stats = nullptr);

// Text stem: x = tok[ids] + pos; h = ln_1(x) -- or, h == nullptr, stats as launch_vision_embed_ln.
hipError_t launch_text_embed_ln(DType dt, const int64_t* ids, const float* tok, const float* pos,
                                const float* ln1_w, const float* ln1_b, float eps, void* x, int x16,
                                void* h, int B, int T, int D, int vocab, hipStream_t s, uint8_t* qs = nullptr,
                                float* stats = nullptr);

// Pool one row per sequence (CLS: ids == nullptr; else first argmax of ids) and LN it.
hipError_t launch_pool_ln(DType dt, const void* x, int x16, const int64_t* ids, int tokens,
                          const float* w, const float* b, float eps, void* out16, int B, int D,
                          hipStream_t s);

// Last-layer compaction: xc[b] = x[b*tokens + pos(b)] (the residual type) and hc[b] = h[same row]
// (16-bit), pos as launch_pool_ln picks it.  x / h and xc / hc must not overlap.
hipError_t launch_gather_pooled(const void* x, int x16, const void* h16, const int64_t* ids, int tokens, void* xc,
                                void* hc16, int B, int D, hipStream_t s);

// Patch rows of the patch-embedding conv: out[b*G*G + p][k] (16-bit, row stride Kp) from
// normalised f32 NCHW (src = A_IMG_F32) or u8 NHWC normalised with mean/std (A_IMG_U8);
// k = ch*P*P + ky*P + kx, zero for Kv <= k < Kp.  G = S / P.
hipError_t launch_patch_rows(DType dt, int src, const void* img, const float* mean, const float* stdv, void* out,
                             int B, int S, int P, int Kv, int Kp, hipStream_t s);

// GPU crop + resize (kernels/resize.hip) of n RGB8 images to u8 NHWC out[n][S][S][3], from
// the host's ResizePlan tables: per image a descriptor (offsets into the raw / tmp byte
// arenas and into the int32 arena holding bounds + fixed-point coefficients).
struct ResizeImage {
  long src, tmp;            // byte offsets: source [H][W][3] in raw, pass-1 output [th][S][3] in tmp
  long h_bounds, h_coef;    // int offsets in ints: [S][2] (first, count), [S][h_ksize]
  long v_bounds, v_coef;    // [S][2] (relative to the pass input rows), [S][v_ksize]
  int W, th, yfirst, h_ksize, v_ksize, need_h, need_v, h_prec, v_prec, pad[3];  // *_prec: fixed-point bits
};
hipError_t launch_resize(const uint8_t* raw, uint8_t* tmp, const int* ints, const ResizeImage* d_imgs, int n,
                         int max_th, int S, uint8_t* out, hipStream_t s);

// Clip facade math (kernels/similarity.hip): out[i][j] = act(fmaf(img[i] . txt[j], scale, bias)),
// act = softmax along axis (1: over labels per image, 0: over images per label), sigmoid, or none.
enum SimAct { SIM_SOFTMAX = 0, SIM_SIGMOID = 1, SIM_LOGITS = 2 };
hipError_t launch_similarity(const float* img, int ni, const float* txt, int nt, int E, float scale, float bias,
                             int activation, int axis, float* out, hipStream_t s);

// out[r] = in[r] / max(||in[r]||_2, 1e-12)
hipError_t launch_l2norm(const float* in, float* out, int B, int E, hipStream_t s);

// f32 -> T16 conversion (weight upload).
hipError_t launch_cast_f32(DType dt, const float* in, void* out, long n, hipStream_t s);
// dst[0 .. bytes) = host-mapped src (16-byte aligned, bytes % 16 == 0), read by a grid of CUs.
hipError_t launch_pull_copy(const void* src_mapped, void* dst, size_t bytes, hipStream_t s);

#ifdef CLIPGPU_GEMM_STAMPS
// Diagnostic build: copy (or clear) the per-block s_memtime stamps of the last GEMM launch.
hipError_t read_gemm_stamps(unsigned long long* host, int nblocks, bool clear);
#endif

// ---- MX-fp8 path (gemm_mx.hip) ---------------------------------------------------------
// An MX-fp8 matrix is OCP e4m3fn bytes [rows][ld] plus E8M0 scale bytes [rows][lds], one per
// 32 consecutive elements of a row: element = e4m3 * 2^(scale - 127).  K % 128 == 0.
struct MxGemmParams {
  const uint8_t* A; long lda; const uint8_t* As; long ldas;  // activations [M][K]
  const uint8_t* W; long ldw; const uint8_t* Ws; long ldws;  // weights [N][K]
  const float* bias;                                         // [N] or nullptr
  void* out; long ldo;     // EPI_STORE16: T16, EPI_RESID / EPI_STORE32: f32, EPI_STOREQ: e4m3 bytes
  uint8_t* outs; long ldos;  // EPI_STOREQ: the output's scales [M][N/32]
  int M, N, K;
  int tile;                // MxTile
  int x16;                 // EPI_RESID: the residual stream `out` is f16 (else f32); the adds are f32
};
enum MxTile {
  MX_TILE_AUTO = 0,
  MX_TILE_256x256 = 1,  // not built: 64x128+ per wave spills (> 256 VGPRs at 2 waves / SIMD; the 4-wave
                        // 128x128-per-wave form spills past 512 with the loop-carried fragment copies)
  MX_TILE_256x128 = 2,  // 8 waves (4x2, 64x64 each), 99 KiB LDS, 1 block / CU
  MX_TILE_128x128 = 3,  // 4 waves (64x64 each), 68 KiB LDS, 2 blocks / CU
  // (round 5: a 4-wave 128x256 with 64x128 per wave at one wave per SIMD -- 387 VGPRs, no spills --
  // measured 0.75-1.0x of this tile at every trunk shape, profiles/r05_mx_sweep.jsonl: not kept)
  MX_TILE_LAST = MX_TILE_128x128,
};
// epi: EPI_STORE16 (act), EPI_RESID, EPI_STORE32, EPI_STOREQ (act); N % 32 == 0.
hipError_t launch_gemm_mx(DType dt, int epi, int act, const MxGemmParams& p, hipStream_t s);
// Rows of f32 (src_dt < 0) or 16-bit (DType) values -> MX-fp8; cols % 32 == 0.
hipError_t launch_quant_rows(int src_dt, const void* src, long ld, uint8_t* q, long ldq, uint8_t* qs, long ldqs,
                             int rows, int cols, hipStream_t s);

}  // namespace clipgpu
