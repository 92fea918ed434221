/*
 * clipgpu — MI355X-native CLIP embedding engine, C ABI.
 *
 * This is the drop-in boundary for the hot path of RuurdBijlsma/clip-embedder-rs
 * (crate open_clip_inference v0.4.0):
 *
 *     image/text -> preprocess/tokenize -> ViT / text transformer -> L2-normalised [B, E]
 *
 * Each entry point names the reference interface it replaces (file:line under the
 * reference tree).  Conventions mirror the reference:
 *   - caller owns every input/output buffer; the engine copies in and out
 *     (Value::from_array + .to_owned(), src/vision.rs:105-113, src/text.rs:153-166);
 *   - return 0 on success, non-zero on error; clipgpu_last_error() gives the
 *     thread-local message (maps to ClipError::Inference / ::Config / ::Io, src/error.rs:9-41);
 *   - an empty batch is an error "Empty batch" (src/vision.rs:121-123);
 *   - one call per handle at a time: each handle serialises its callers with an internal
 *     mutex (the reference's RwLock write lock, src/vision.rs:107, src/text.rs:155);
 *     separate handles are independent (duplicate(), src/vision.rs:86-91).
 * No torch / ndarray / ort types cross this boundary: plain pointers and sizes only.
 */
#ifndef CLIPGPU_H
#define CLIPGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CLIPGPU_ABI_VERSION 4

enum clipgpu_status {
  CLIPGPU_OK = 0,
  CLIPGPU_ERR_INVALID = 1,   /* bad argument / shape          -> ClipError::Inference / Shape */
  CLIPGPU_ERR_CONFIG = 2,    /* model dir / config problem    -> ClipError::Config / MissingModelFile */
  CLIPGPU_ERR_IO = 3,        /* file system                   -> ClipError::Io */
  CLIPGPU_ERR_DEVICE = 4,    /* HIP / RCCL failure            -> ClipError::Inference */
  CLIPGPU_ERR_TOKENIZER = 5  /* tokenizer failure             -> ClipError::Tokenizer */
};

enum clipgpu_tower { CLIPGPU_TOWER_VISION = 0, CLIPGPU_TOWER_TEXT = 1 };
/* CLIPGPU_DTYPE_FP8: the fp8 weight path of BASELINE configs[4] -- the QKV, c_fc and c_proj
 * GEMMs run as MX-fp8 (OCP e4m3 weights and activations, E8M0 scale per 32 K-elements,
 * block-scaled MFMA); attention, out_proj, stems and heads run in bf16.  Needs width and MLP
 * width % 128 == 0.  Lossy: the embeddings do not meet the bf16 path's cosine bar. */
enum clipgpu_dtype { CLIPGPU_DTYPE_BF16 = 0, CLIPGPU_DTYPE_F16 = 1, CLIPGPU_DTYPE_FP8 = 2 };

typedef struct clipgpu_engine clipgpu_engine;       /* one tower on one or more GPUs (== one OnnxSession) */
typedef struct clipgpu_tokenizer clipgpu_tokenizer; /* CLIP BPE tokenizer (== tokenizers::Tokenizer) */

/* Thread-local message for the last failed call on this thread ("" if none). */
const char* clipgpu_last_error(void);
int clipgpu_abi_version(void);
/* sha256 fingerprint of the sources this library was built from (binary provenance; the
 * Python host refuses a library whose fingerprint differs from its tree's). */
const char* clipgpu_build_source_hash(void);

/* ---- engine lifecycle ----------------------------------------------------------------
 * Replaces OnnxSession::new (src/onnx.rs:13-30) as called by VisionEmbedder::from_local_dir
 * (src/vision.rs:58-84) / TextEmbedder::from_local_dir (src/text.rs:54-101).
 * model_dir must hold open_clip_config.json and model_config.json plus a weight source, in
 * this order of preference: open_clip_model.safetensors; the reference's own export
 * visual.onnx / text.onnx (+ .onnx.data external data, pull_onnx.py:170-195; initializers by
 * open_clip name, with or without the "model." wrapper prefix); or clipgpu_synthetic.json
 * {"seed": N} (seeded weights).
 * device_ids/n_devices: the GPUs this handle replicates the weights onto (data-parallel
 * batch sharding across them); NULL/0 = device 0.  max_batch: rows per device per launch
 * (larger batches are processed in chunks).
 * Speed (never the output bits): the GEMM tiles and lane count come from a table measured on
 * MI355X (engine.hip table_tiles / table_lanes) for one lane's token rows at max_batch: the
 * measured regimes are >= 2048 rows per lane (ViT-B/32 vision 256, text 1024, SO400M 128, H/14
 * 64 per GPU); smaller max_batch uses the shape heuristic (skinny kernel at <= 256 rows), and
 * clipgpu_options.tuning = 1 times the candidates at creation for any other batch. */
int clipgpu_create(const char* model_dir, int tower, const int* device_ids, int n_devices, int dtype,
                   int max_batch, clipgpu_engine** out);
void clipgpu_destroy(clipgpu_engine* e);

/* Per-engine options (clipgpu_create_ex; clipgpu_create == clipgpu_create_ex with opts = NULL).
 * The reference builds each tower's session with its own SessionBuilder settings
 * (src/onnx.rs:13-30); these are this engine's equivalents, per handle, so one process can hold
 * e.g. an fp8 vision tower beside a bf16 text tower with different MX splits. */
#define CLIPGPU_MX_QKV 1u  /* fp8 engines: the QKV projection runs as an MX-fp8 GEMM */
#define CLIPGPU_MX_FC 2u   /* c_fc */
#define CLIPGPU_MX_PROJ 4u /* c_proj (needs CLIPGPU_MX_FC: c_fc's epilogue quantizes the hidden rows) */
#define CLIPGPU_RESIDUAL_F32 1
#define CLIPGPU_RESIDUAL_F16 2
typedef struct clipgpu_options {
  uint32_t struct_size; /* sizeof(clipgpu_options) (set by clipgpu_options_init); an older caller's
                           smaller struct keeps the defaults of the fields it does not have */
  uint32_t mx_sites;    /* fp8 engines: CLIPGPU_MX_* bits; 0 = default (all three) */
  int32_t lanes;        /* concurrent sub-batch lanes per device, 1..4; 0 = the tile table's choice */
  int32_t tuning;       /* 0 = GEMM tiles and lanes from the committed MI355X tile table
                           (deterministic, default); 1 = time the candidates at creation, per site and
                           then over whole forwards; 2 = the per-site timing only (the choice then
                           depends on the timings; it never changes the output bits) */
  int32_t communicator; /* handles over > 1 distinct devices: 1 = create the RCCL communicator at
                           creation; 0 (default) = on the first gathered call */
  /* ---- ABI v3 (round 4): every engine behaviour is a field here; the library reads no
   * environment variables.  0 is the default everywhere. */
  int32_t graphs;       /* 0 / 1 = replay each forward as a captured hipGraph (default); -1 = launch
                           the kernels directly (bit-identical) */
  int32_t prune_last;   /* 0 / 1 = the last layer runs on the pooled rows only (default; bit-identical);
                           -1 = on every token */
  int32_t trim_text;    /* 0 / 1 = host-id text batches run on their first max(EOT index) + 1 tokens
                           (default; bit-identical); -1 = on the full context */
  int32_t gemm_tiles[4]; /* GEMM tile per trunk site (qkv, out_proj, c_fc, c_proj): 0 = the table's
                           (or tuner's) choice, -1 = the shape heuristic, else a GemmTile id the library
                           builds (csrc/kernels/kernels.hpp kGemmTiles; speed only, never the bits) */
  int32_t patch_tile;   /* the vision patch-embedding GEMM's tile, as gemm_tiles */
  uint32_t mx_layers;   /* fp8 engines: bit l set = layer l runs its MX sites in MX-fp8, the other layers
                           run every GEMM in bf16; 0 = every layer (default).  Layers 0..31 only (a
                           tower's layers >= 32 run bf16 under a non-zero mask); a bit at or beyond the
                           tower's layer count is refused (CLIPGPU_ERR_INVALID) */
  /* ---- ABI v4 (round 5) */
  int32_t residual;     /* storage of the residual stream x: 1 = f32; 2 = f16 (half the bytes of x's two
                           read-modify-writes and two LayerNorm reads per layer; every add into x and every
                           LayerNorm statistic stays f32; CLIP-family engines of every dtype, SigLIP
                           CLIPGPU_ERR_INVALID); 0 = the default: f16 where it applies, else f32.  f16 holds
                           |x| <= 65504 (a larger value is stored as inf); CLIP / DFN residual streams stay in
                           the hundreds (tests/test_gpu_parity.py test_massive_residual_channels_parity):
                           choose 1 for a checkpoint whose stream exceeds that range */
  int32_t ln_fold;      /* ln_1 / ln_2 folded into the QKV / c_fc GEMMs (f16 residual stream only): the GEMM
                           reads x itself with W' = W diag(gamma) in f16 and applies each row's mean / rstd
                           and bias + W beta in its epilogue; the rows' (mean, rstd) come from a statistics-only
                           pass (8 bytes per row) instead of a normalised copy of x.  0 = the default: on where
                           it applies (bf16 / f16 engines, residual f16, QuickGELU / GELU MLP); 1 = on
                           (CLIPGPU_ERR_INVALID where it does not apply); -1 = off (LayerNorm kernels + bf16 /
                           f16 GEMMs) */
} clipgpu_options;
/* Fills *opts with the defaults. */
int clipgpu_options_init(clipgpu_options* opts);
int clipgpu_create_ex(const char* model_dir, int tower, const int* device_ids, int n_devices, int dtype,
                      int max_batch, const clipgpu_options* opts, clipgpu_engine** out);
/* The engine's resolved choices: tiles[4] = GemmTile per trunk site (qkv, out_proj, c_fc, c_proj),
 * *lanes = concurrent lanes of a device-side forward, *mx_sites = CLIPGPU_MX_* bits in use. */
int clipgpu_engine_info(const clipgpu_engine* e, int tiles[4], int* lanes, uint32_t* mx_sites);

int clipgpu_embed_dim(const clipgpu_engine* e);      /* E */
int clipgpu_input_size(const clipgpu_engine* e);     /* vision: image_size S; text: context length T */
int clipgpu_num_devices(const clipgpu_engine* e);

/* ---- vision forward ------------------------------------------------------------------
 * Replaces session.run(pixel_values) + extract in VisionEmbedder::embed_images
 * (src/vision.rs:100-117).  nchw: [B,3,S,S] f32, already normalised (preprocess_batch
 * output, src/vision.rs:119-135).  out: [B,E] f32 row-major, L2-normalised. */
int clipgpu_embed_pixels(clipgpu_engine* e, const float* nchw, int64_t B, int64_t S, float* out);

/* Device-side-normalise variant: nhwc u8 [B,S,S,3] (already resized/cropped), mean/std
 * applied on the GPU exactly as normalize_pixels (src/vision.rs:235-259). */
int clipgpu_embed_u8(clipgpu_engine* e, const uint8_t* nhwc, int64_t B, int64_t S, const float mean[3],
                     const float std[3], float* out);

/* ---- caller-registered host buffers ------------------------------------------------------
 * The reference's embed_images / embed_texts hand host arrays to the session (src/vision.rs:102-113,
 * src/text.rs:150-166).  By default the host-buffer entry points stage them through the handle's
 * pinned buffers (a host copy, then the PCIe DMA).  A caller that reuses its buffers can pin them once
 * (hipHostRegister, mapped and portable): an embed_* call whose whole input (or output) lies inside a
 * registered range then DMAs straight from (into) it, skipping the host copy; the batch still moves
 * in one chunk per lane, so the first chunk's transfer is what is exposed before the forward starts.
 * Results are bit-identical either way.  Process-wide; the caller keeps the memory alive, and
 * unregisters it only when no embed_* call is using it, before freeing it.  Ranges may not overlap. */
int clipgpu_host_register(void* ptr, size_t bytes);
int clipgpu_host_unregister(void* ptr);

/* ---- text forward ---------------------------------------------------------------------
 * Replaces session.run(input_ids [, attention_mask]) in TextEmbedder::embed_texts
 * (src/text.rs:148-169).  ids: [B,T] int64; mask may be NULL (the exported text graph has
 * no mask input, pull_onnx.py:296-302; it is accepted and ignored, as the reference does
 * when the graph lacks "attention_mask", src/text.rs:156-161).  The batch runs on its first
 * max(EOT index)+1 tokens (at least 16; bit-identical to the full context under causal
 * attention and argmax pooling; clipgpu_options.trim_text = -1 disables). */
int clipgpu_embed_tokens(clipgpu_engine* e, const int64_t* ids, const int64_t* mask, int64_t B, int64_t T,
                         float* out);

/* ---- device-resident entry points (benchmarks, zero-copy pipelines) ----------------------
 * Inputs/outputs are device pointers on the handle's first device; work is ordered on
 * `stream` (a hipStream_t; NULL = the legacy default stream, as in HIP's own APIs, which is
 * also torch's default stream) and the call returns without synchronising: work enqueued on
 * `stream` before the call is complete before the forward reads its input, and work enqueued
 * after it sees the finished embeddings.  The forward itself runs as a hipGraph on the
 * handle's stream, forked from and joined back to `stream` by events.  B <= max_batch. */
int clipgpu_embed_pixels_device(clipgpu_engine* e, const float* d_nchw, int64_t B, float* d_out, void* stream);
int clipgpu_embed_u8_device(clipgpu_engine* e, const uint8_t* d_nhwc, int64_t B, const float mean[3],
                            const float std[3], float* d_out, void* stream);
int clipgpu_embed_tokens_device(clipgpu_engine* e, const int64_t* d_ids, int64_t B, float* d_out, void* stream);

/* Decoded images straight to embeddings, crop/resize on the GPU (a3-a7 on the device).
 * Replaces preprocess_batch + session.run in VisionEmbedder::embed_images
 * (src/vision.rs:100-162): images[i] is [heights[i]][widths[i]][3] u8 (DynamicImage::to_rgb8
 * layout, any size); the model folder's preprocess_cfg (interpolation, resize_mode, mean,
 * std; src/config.rs:49-64) applies.  The GPU resize uses the host resize's fixed-point
 * tables, so results are bit-identical to clipgpu_preprocess_batch + clipgpu_embed_pixels.
 * out: [n,E] f32, L2-normalised. */
int clipgpu_embed_images_rgb8(clipgpu_engine* e, const uint8_t* const* images, const int* widths, const int* heights,
                              int64_t n, float* out);

/* ---- host preprocessing (src/vision.rs:119-259) ----------------------------------------
 * rgb: [h][w][3] u8 (DynamicImage::to_rgb8 layout).  Resize with the crop box of
 * resize_with_fast_image_resize (src/vision.rs:164-198): unless resize_mode == "squash",
 * the centred min(w,h) square; interpolation "bicubic" (CatmullRom) / "bilinear" / other
 * (nearest).  Then normalize_pixels (src/vision.rs:235-259) into out_chw [3][size][size]. */
int clipgpu_preprocess_rgb8(const uint8_t* rgb, int width, int height, int size, const char* interpolation,
                            const char* resize_mode, const float mean[3], const float std[3], float* out_chw);
/* Resize/crop only: out_rgb [size][size][3] u8. */
int clipgpu_resize_rgb8(const uint8_t* rgb, int width, int height, int size, const char* interpolation,
                        const char* resize_mode, uint8_t* out_rgb);
/* Batch preprocess with a host thread pool (preprocess_batch's rayon loop, src/vision.rs:128-132):
 * images[i] is [heights[i]][widths[i]][3] u8; out: [n][3][size][size]. */
int clipgpu_preprocess_batch(const uint8_t* const* images, const int* widths, const int* heights, int64_t n,
                             int size, const char* interpolation, const char* resize_mode, const float mean[3],
                             const float std[3], float* out);
/* The crate's non-default resize, resize_with_image (src/vision.rs:200-233; the build without the
 * `fast_image_resize` feature): the image crate 0.25.9's imageops::resize (f32 separable filter,
 * vertical pass then horizontal, CatmullRom / Triangle / Nearest) to round(W*s) x round(H*s),
 * s = size / min(W, H), then crop_imm at the rounded centre offsets ("squash": resize_exact to
 * size x size).  Same arguments and outputs as clipgpu_resize_rgb8 / clipgpu_preprocess_batch. */
int clipgpu_resize_rgb8_image(const uint8_t* rgb, int width, int height, int size, const char* interpolation,
                              const char* resize_mode, uint8_t* out_rgb);
int clipgpu_preprocess_batch_image(const uint8_t* const* images, const int* widths, const int* heights, int64_t n,
                                   int size, const char* interpolation, const char* resize_mode, const float mean[3],
                                   const float std[3], float* out);

/* ---- tokenizer (src/text.rs:62-139) ----------------------------------------------------
 * Loads a HF tokenizers CLIP tokenizer.json (BPE + ByteLevel, </w> suffix) and applies
 * with_padding(Fixed(context_length), pad_id) + with_truncation(max_length=context_length)
 * as TextEmbedder::from_local_dir does (src/text.rs:70-85).  pad_id < 0: look up "<pad>"
 * in the vocab (src/text.rs:70-73). */
int clipgpu_tokenizer_create(const char* tokenizer_json, int context_length, int64_t pad_id,
                             clipgpu_tokenizer** out);
void clipgpu_tokenizer_destroy(clipgpu_tokenizer* t);
/* texts: n UTF-8 strings; lengths[i] = byte length of texts[i] (like a Rust &str, may contain NUL),
 * or lengths == NULL for NUL-terminated strings.  lowercase != 0 applies str::to_lowercase first
 * (tokenizer_needs_lowercase, src/text.rs:115-117).  ids, mask: [n][context_length]. */
int clipgpu_tokenize(clipgpu_tokenizer* t, const char* const* texts, const int64_t* lengths, int64_t n,
                     int lowercase, int64_t* ids, int64_t* mask);
/* Token id of a vocab string, or -1. */
int64_t clipgpu_tokenizer_token_id(const clipgpu_tokenizer* t, const char* token);
int64_t clipgpu_tokenizer_vocab_size(const clipgpu_tokenizer* t);

/* ---- Clip facade math for many images x many labels -------------------
 * The src/clip.rs:79-185 arithmetic on the GPU: logits[i][j] = dot(img[i], txt[j]).mul_add(
 * logit_scale, logit_bias) (ModelConfig defaults 1.0 / 0.0 are the caller's), then
 *   activation CLIPGPU_SIM_SOFTMAX: max-subtracted softmax along `axis` -- 1 = over the labels
 *     of each image (classify, :92-132), 0 = over the images of each label (rank_images,
 *     :134-170);  CLIPGPU_SIM_SIGMOID: elementwise sigmoid (activation_function "sigmoid");
 *   CLIPGPU_SIM_LOGITS: the logits themselves (compare, :79-90).
 * img [n_img][E], txt [n_txt][E] f32 (the embed_* outputs); out [n_img][n_txt] f32; E % 16 == 0.
 * Host-buffer form on GPU `device`; the _device form takes device pointers and a stream.
 * (The descending sort of classify / rank_images stays on the host.) */
enum clipgpu_sim_activation { CLIPGPU_SIM_SOFTMAX = 0, CLIPGPU_SIM_SIGMOID = 1, CLIPGPU_SIM_LOGITS = 2 };
int clipgpu_similarity(int device, const float* img, int64_t n_img, const float* txt, int64_t n_txt, int64_t E,
                       float logit_scale, float logit_bias, int activation, int axis, float* out);
int clipgpu_similarity_device(const float* d_img, int64_t n_img, const float* d_txt, int64_t n_txt, int64_t E,
                              float logit_scale, float logit_bias, int activation, int axis, float* d_out,
                              void* stream);

/* ---- data-parallel sharding + the RCCL all-gather (north_star: "batches shard
 * data-parallel across the 8 GPUs of one node with an RCCL all-gather over xGMI only for the final
 * embedding matrix").  The reference has no multi-device path: embed_images / embed_texts
 * (src/vision.rs:100-117, src/text.rs:148-169) keep their signatures; these entry points are
 * what a multi-GPU caller of them binds.
 * Communicator: a handle created over n > 1 DISTINCT devices owns one (ncclCommInitAll, rank i =
 * device_ids[i]), created on its first gathered call (or at creation with
 * clipgpu_options.communicator = 1), so creation and the host-buffer entry points never depend
 * on RCCL; a one-device handle in a one-process-per-GPU deployment joins one with
 * clipgpu_comm_init_rank (rank 0 calls clipgpu_comm_unique_id and sends the 128 bytes to every
 * rank out of band; every rank then calls init_rank, collectively).  clipgpu_comm_info gives
 * (nranks, first rank of this handle); nranks 0 = no communicator.
 * Gathered forward: rows[nranks] = every rank's block size (identical on every rank); per LOCAL
 * device i (rank = first rank + i): d_in[i] = that rank's block on device i (f32 NCHW normalised
 * pixels / i64 ids [rows][T]), d_out[i] = [sum rows][E] f32 on device i, streams[i] (a NULL entry, or
 * a NULL array: device i's legacy default stream, as for the single-device *_device entry points).
 * Each rank embeds its block into its slot, then one collective
 * (in-place ncclAllGather for equal blocks; one ncclBroadcast per block otherwise) leaves the
 * whole matrix in rank order on every device.  Stream-ordered; collective over all ranks. */
int clipgpu_comm_unique_id(uint8_t* id /* [128] */);
int clipgpu_comm_init_rank(clipgpu_engine* e, const uint8_t* id /* [128] */, int nranks, int rank);
int clipgpu_comm_info(const clipgpu_engine* e, int* nranks, int* rank0);
int clipgpu_embed_pixels_gather_device(clipgpu_engine* e, const float* const* d_nchw, const int64_t* rows,
                                       float* const* d_out, void* const* streams);
int clipgpu_embed_tokens_gather_device(clipgpu_engine* e, const int64_t* const* d_ids, const int64_t* rows,
                                       float* const* d_out, void* const* streams);

/* ---- Clip facade scores on the host, the reference's f32 arithmetic bit for bit -----------
 * src/clip.rs:79-185 as the crate computes it (ndarray 0.17 without BLAS, Cargo.toml:14):
 * out[i] = unrolled_dot(embs[i], query).mul_add(logit_scale, logit_bias) -- ndarray's
 * eight-accumulator numeric_util::unrolled_dot, one fused multiply-add -- then
 *   CLIPGPU_SIM_SOFTMAX: max (f32::max fold) -> exp(x - max) -> sequential f32 sum -> x / sum
 *     over the n scores (classify :92-132 with embs = label embeddings, query = the image;
 *     rank_images :134-170 with embs = image embeddings, query = the text);
 *   CLIPGPU_SIM_SIGMOID: 1 / (1 + exp(-l)) (:181-185);  CLIPGPU_SIM_LOGITS: the logits (compare,
 *     :79-90, n = 1).
 * embs [n][E], query [E], out [n] f32; no GPU involved.  n == 0 -> "Empty batch". */
int clipgpu_facade_scores(const float* embs, int64_t n, const float* query, int64_t E, float logit_scale,
                          float logit_bias, int activation, float* out);

/* ---- live kernel timing -------------------------------------------------------------------
 * Records HIP events around every launch whose category bit is set in `mask` (on the launch
 * stream), for the device-resident entry points.  Categories: 0 patch_embed, 1 stem_ln, 2 qkv,
 * 3 attention, 4 out_proj, 5 layernorm, 6 c_fc, 7 c_proj, 8 head, 9 last_layer (the pruned
 * last layer's gather, out_proj, ln_2, c_fc and c_proj at M = batch).  enable() resets totals;
 * read() waits for the recorded events and returns the summed ms and launch count.  While a
 * mask is set, a batch's concurrent sub-batch lanes run one after another on the launch
 * stream (same launches, no overlap), so each event pair times one kernel alone -- unless the
 * mask also has CLIPGPU_PROFILE_CONCURRENT: then the lanes stay concurrent (no graph replay) and
 * each GEMM's event pair times its launch beside the other lane's kernels, as in the timed step. */
#define CLIPGPU_PROFILE_CONCURRENT 0x80000000u
int clipgpu_profile_enable(clipgpu_engine* e, unsigned mask);
int clipgpu_profile_read(clipgpu_engine* e, int category, double* total_ms, int64_t* launches);
const char* clipgpu_profile_category_name(int category);

/* ---- test hooks --------------------------------------------------------------------------
 * The seeded weight generator shared with the oracle (bit-exact). */
int clipgpu_synth_tensor(uint64_t seed, const char* name, double std, double offset, float* out, int64_t n);

#ifdef __cplusplus
}
#endif

#endif /* CLIPGPU_H */
