/*
 * clipgpu kernel-level test hooks (not part of the drop-in surface).
 *
 * Each hook uploads host f32 buffers, runs ONE gfx950 kernel of the hot path on
 * device 0, and copies the result back, so tests/ can check every kernel in
 * isolation against a numpy fp32/fp64 reference of the same op.  All return 0 on
 * success (message via clipgpu_last_error()).  dtype: CLIPGPU_DTYPE_BF16 / _F16.
 */
#ifndef CLIPGPU_TESTING_H
#define CLIPGPU_TESTING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* out[M][N] = act(A[M][K] . W[N][K]^T + bias[N]) (act: 0 none, 1 quick_gelu, 2 gelu, 3 gelu_tanh).
 * mode 0: 16-bit output (returned as f32); mode 1: residual (out = resid + ...); mode 2: f32 output;
 * mode 3: residual on an f16 stream (resid rounded to f16 on upload, the f16 result widened to f32).
 * bias and resid may be NULL.  CLIPGPU_TEST_TILE = a GemmTile id the library builds (kernels.hpp
 * kGemmTiles; 0 auto, 100 skinny, 101 the skinny kernel's general form) forces the tile; shapes the pipelined tiles do not take (K = 64,
 * 16-bit rows not a multiple of 8 elements) run the skinny kernel's general form whatever the tile (test hooks only: the engine reads no environment). */
int clipgpu_test_gemm(int dtype, int mode, int act, int64_t M, int64_t N, int64_t K, const float* A,
                      const float* W, const float* bias, const float* resid, float* out);
/* The LayerNorm-folded GEMM (EPI_LNF): out[m][n] = act(rstd_m (x W'^T - mean_m cs)[m][n] + bias[n]) with
 * x [M][K] and wf [N][K] rounded to f16 on upload, mean / rstd of each row of x (eps; launch_ln_stats,
 * K <= 1280), the output in dtype (bf16 / f16), widened to f32.  tile: a built GemmTile, 0 = the
 * launcher's choice, 100 = skinny. */
int clipgpu_test_gemm_lnf(int dtype, int act, int64_t M, int64_t N, int64_t K, const float* x, const float* wf,
                          const float* cs, const float* bias, float eps, int tile, float* out);

/* Cap the rows of one GEMM launch of launch_gemm's row-chunked path (0 = off: only the 2^31-byte operand
 * limit chunks), process-wide, for every GEMM launched (or graph captured) afterwards: the chunked path
 * of large batches runs at test sizes.  Chunking is bit-invisible. */
int clipgpu_test_gemm_chunk_rows(int64_t rows);

/* qkv: [B*N][3*D] f32 (rounded to 16-bit on upload), D = H * HD (HD in {64, 72, 80}); out: [B*N][D]. */
int clipgpu_test_attention(int dtype, int64_t B, int64_t N, int64_t H, int64_t HD, int causal, const float* qkv,
                           float* out);

/* out[r] = LN(x[r]) (16-bit output returned as f32). */
int clipgpu_test_layernorm(int dtype, int64_t rows, int64_t D, float eps, const float* x, const float* w,
                           const float* b, float* out);

/* Patch-embedding stem from normalised f32 NCHW pixels (mode 0) or u8 NHWC (mode 1), as the
 * engine runs it (patch rows, then the row GEMM with the patch epilogue):
 * x_out[B*(G*G+1)][D]: rows of patch tokens = conv + pos (CLS rows untouched = 0). */
int clipgpu_test_patch_embed(int dtype, int mode, int64_t B, int64_t S, int64_t P, int64_t D, const void* pixels,
                             const float mean[3], const float std[3], const float* conv_w, const float* pos,
                             float* x_out);

/* The GPU crop/resize alone (kernels/resize.hip): out [n][size][size][3] u8, to compare with
 * clipgpu_resize_rgb8 (host) bit for bit. */
int clipgpu_test_resize_rgb8_gpu(const uint8_t* const* images, const int* widths, const int* heights, int64_t n,
                                 int size, const char* interpolation, const char* resize_mode, uint8_t* out);

/* The cross-lane reduction helpers (DPP row rotations + permlane swaps) on one wave: out[k*64 + lane]
 * for k = 0 wave_sum, 1 wave_max, 2 x + x[lane^16], 3 x + x[lane^32], 4 row-of-16 sum, 5 row-of-16 max,
 * 6 / 7 the two results of the raw permlane16 swap of (x, x). */
int clipgpu_test_lane_reduce(const float* in64, float* out512);

/* The staged 16-bit patch rows alone: rows_out[B*G*G][Kp] (as f32), Kp = 3*P*P rounded up to 64. */
int clipgpu_test_patch_rows(int dtype, int mode, int64_t B, int64_t S, int64_t P, const void* pixels,
                            const float mean[3], const float std[3], float* rows_out);

/* Device-resident GEMM timing (random operands): `iters` back-to-back launches of the same
 * GEMM as the engine issues it (epi: 0 store16 (+act), 1 residual f32, 2 store32, 3 residual f16), tile: a GemmTile
 * id (kernels.hpp; 0 auto).  Returns the mean µs per launch (HIP events). */
int clipgpu_test_gemm_bench(int dtype, int epi, int act, int64_t M, int64_t N, int64_t K, int tile, int iters,
                            double* us_per_launch);
/* Blocks of one launch of GEMM tile `tile` (0 auto) at M x N x K (row operands): the persistent grid
 * the launcher uses (one CU's resident blocks x CUs, or the tile count when smaller).  No GPU needed
 * (a host without one counts 256 CUs). */
int clipgpu_test_gemm_grid(int tile, int64_t M, int64_t N, int64_t K, int* grid);
/* As clipgpu_test_gemm_bench with row pitches lda >= K, ldw >= K (elements, multiples of 8). */
int clipgpu_test_gemm_bench_ld(int dtype, int epi, int act, int64_t M, int64_t N, int64_t K, int64_t lda,
                               int64_t ldw, int tile, int iters, double* us_per_launch);

/* Host copy rate: one `bytes` copy from page-aligned malloc'd memory, `iters` times, µs per copy.
 * mode 0: std::memcpy into malloc'd memory; 1: the copy pool (pool_memcpy) into it; 2 / 3: the same
 * into pinned hipHostMalloc memory (the host path's staging). */
int clipgpu_test_host_copy(int64_t bytes, int mode, int iters, double* us_per_copy);
/* Installs a SIGSEGV / SIGABRT handler that prints the faulting thread's frames as object + offset
 * (diagnostics for GPU-box runs), then re-raises. */
int clipgpu_test_install_crash_handler(void);
/* Shader-clock probe (bench.py's per-window clock): launches ONE wave on `stream` (a hipStream_t, NULL =
 * the legacy default stream) that sleeps for duration_us of wall time (s_memrealtime, 100 MHz) and writes
 * d_out[0] = shader-clock ticks (s_memtime) and d_out[1] = 100 MHz ticks elapsed over that span (device
 * uint64 buffer of 2): MHz = 100 * d_out[0] / d_out[1] (MI355X_MICROARCH.md, DVFS give-back item 6).
 * Asynchronous.  bench.py launches it right after a timed window: resident beside a forward, its wave
 * keeps one CU from hosting the one-block-per-CU GEMMs. */
/* Host-to-device copy rate: `bytes` from a pinned mapped host buffer into device memory, mode 0 = one
 * hipMemcpyAsync (SDMA), 1 = a copy kernel reading through the host mapping, 2 = the halves as two
 * SDMA copies on two streams, 3 = the first half by the copy kernel beside the second half's SDMA
 * copy; + 4: the host buffer is page-aligned malloc'd memory registered (hipHostRegister, as
 * clipgpu_host_register) instead of hipHostMalloc'd.  Returns the mean µs per copy (HIP events). */
int clipgpu_test_h2d_bench(int64_t bytes, int mode, int iters, double* us_per_copy);
int clipgpu_test_clock_probe(void* stream, int64_t duration_us, uint64_t* d_out);

/* Device-resident attention timing (random 16-bit qkv): mean µs per launch_attention over `iters`. */
int clipgpu_test_attention_bench(int dtype, int64_t B, int64_t N, int64_t H, int64_t HD, int causal, int iters,
                                 double* us_per_launch);

/* MX-fp8 (OCP e4m3fn bytes + one E8M0 scale byte per 32 consecutive elements of a row; element =
 * e4m3 * 2^(scale - 127)).  Quantizer: in[rows][cols] f32 -> q[rows][cols], qs[rows][cols/32];
 * cols % 32 == 0. */
int clipgpu_test_quant_rows(int64_t rows, int64_t cols, const float* in, uint8_t* q, uint8_t* qs);

/* LayerNorm with the MX-fp8 output the fp8 trunk feeds its MX GEMMs (D % 32 == 0). */
int clipgpu_test_layernorm_mx(int64_t rows, int64_t D, float eps, const float* x, const float* w, const float* b,
                              uint8_t* q, uint8_t* qs);

/* MX-fp8 GEMM on given MX operands A (Aq [M][K], As [M][K/32]) and W (Wq [N][K], Ws [N][K/32]):
 * mode 0: act(A.W^T + bias) as 16-bit (returned as f32 in out); 1: out = resid + A.W^T + bias (f32);
 * 2: f32 A.W^T + bias; 3: MX-fp8 of act(A.W^T + bias) into outq [M][N] / outs [M][N/32].
 * K % 128 == 0, N % 32 == 0; CLIPGPU_TEST_TILE picks the MxTile (0 auto, 2 256x128, 3 128x128). */
int clipgpu_test_gemm_mx(int dtype, int mode, int act, int64_t M, int64_t N, int64_t K, const uint8_t* Aq,
                         const uint8_t* As, const uint8_t* Wq, const uint8_t* Ws, const float* bias,
                         const float* resid, float* out, uint8_t* outq, uint8_t* outs);

/* Device-resident MX GEMM timing (random operands quantized on the device), epi as mode above. */
int clipgpu_test_gemm_mx_bench(int epi, int act, int64_t M, int64_t N, int64_t K, int tile, int iters,
                               double* us_per_launch);

/* Host only (no GPU): the f32 parameter `name` (open_clip state-dict name) of one tower as
 * clipgpu_create would load it from model_dir (safetensors / visual|text.onnx / synthetic);
 * n = element count. */
int clipgpu_test_read_weights(const char* model_dir, int tower, const char* name, float* out, int64_t n);

/* GEMM tile chosen per trunk call site of an engine (0 qkv, 1 out_proj, 2 c_fc, 3 c_proj): a GemmTile
 * id (kernels.hpp), 0 = the shape heuristic; fp8 engines report MxTile ids at their MX sites (2 256x128,
 * 3 128x128).  clipgpu_options.gemm_tiles pins them. */
struct clipgpu_engine;
int clipgpu_test_engine_tiles(const struct clipgpu_engine* e, int tiles[4]);
/* Concurrent sub-batches the engine's device-side forwards run (the creation-time tuning's pick,
 * or clipgpu_options.lanes). */
int clipgpu_test_engine_lanes(const struct clipgpu_engine* e, int* dev_lanes);
/* The residual stream's resolved storage (CLIPGPU_RESIDUAL_F32 / _F16) and whether ln_1 / ln_2 are
 * folded into the QKV / c_fc GEMMs (*ln_fold = 1; clipgpu_options.ln_fold; ln_fold may be NULL). */
int clipgpu_test_engine_residual(const struct clipgpu_engine* e, int* residual, int* ln_fold);
/* The host-buffer vision path's chunk plan (tools/host_plan_ab.py): n_chunks (1..4) chunks of a
 * max_batch round cut at bounds[0 .. n_chunks - 2]; n_chunks = 0 restores the default
 * (engine.hip host_chunks).  copy_stream must be 0 or 1 (round 6 removed the schedule variants it
 * used to select; DESIGN.md §10 keeps their measurements).  Speed only, never the bits. */
int clipgpu_test_host_plan(struct clipgpu_engine* e, int n_chunks, const int* bounds, int copy_stream);
/* on != 0: clipgpu_embed_images_rgb8 sends batches of image_size x image_size images through the GPU
 * resize path too (by default they take the u8 host path: their resize plan is the identity).  The
 * test of the identity route compares the two. */
int clipgpu_test_rgb8_resize_always(struct clipgpu_engine* e, int on);
/* Gathered calls of this handle take the ragged branch (one ncclBroadcast per block) even when
 * every block has the same size (on != 0), so a one-rank or equal-shard run exercises it. */
int clipgpu_test_force_broadcast(struct clipgpu_engine* e, int on);
/* A handle without a communicator takes the multi-device handle's lazy path: a clique over its
 * replicas' distinct devices, created (ncclCommInitAll) by the first gathered call. */
int clipgpu_test_comm_lazy(struct clipgpu_engine* e);
/* The launches recorded by clipgpu_profile_enable as a timeline: up to n_max entries of start / end
 * (ms from the first recorded start), category (clipgpu_profile_category_name) and lane (the device
 * lane stream index, -1 for another stream); *n_out = the number recorded.  Consumes the records as
 * clipgpu_profile_read does (their times then count in its totals). */
int clipgpu_test_profile_timeline(struct clipgpu_engine* e, int64_t n_max, double* t0, double* t1, int* cat,
                                  int* lane, int64_t* n_out);
/* The host-side plan of a gathered call (no GPU): off[0..nranks] = first output row of each rank's
 * block (off[nranks] = total rows), *equal = 1 when every block has the same size.  Errors as the
 * gathered entry points: a negative count, or zero rows in all ("Empty batch"). */
int clipgpu_test_gather_plan(int nranks, const int64_t* rows, int64_t* off, int* equal);

#ifdef __cplusplus
}
#endif

#endif /* CLIPGPU_TESTING_H */
