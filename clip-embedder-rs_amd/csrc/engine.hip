// clipgpu engine: one tower (vision or text) replicated on one or more GPUs.
//
// Replaces the ONNX Runtime session (src/onnx.rs:7-47) that the reference builds
// per tower and runs in VisionEmbedder::embed_images (src/vision.rs:100-117) and
// TextEmbedder::embed_texts (src/text.rs:148-169).  Weights are uploaded once per
// device (16-bit matrices for MFMA, f32 for LayerNorm/bias/embeddings) into one
// arena; activations live in a persistent per-device workspace sized for
// max_batch, so a forward performs no allocation and can be captured in a
// hipGraph.  Multi-device handles shard the batch into contiguous row blocks,
// one host worker thread and one stream per device.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <vector>

#include "../../include/clipgpu.h"
#include "../../include/clipgpu_testing.h"
#include "bounce.hpp"
#include "host/api_util.hpp"
#include "host/copy_pool.hpp"
#include "host/json.hpp"
#include "host/model.hpp"
#include "host/resize_plan.hpp"
#include "kernels/common.hpp"
#include "kernels/kernels.hpp"

namespace clipgpu {

#define NCCL_CHECK(expr)                                                                            \
  do {                                                                                              \
    ncclResult_t _r = (expr);                                                                       \
    if (_r != ncclSuccess)                                                                          \
      throw ClipErr(CLIPGPU_ERR_DEVICE, std::string("RCCL error: ") + ncclGetErrorString(_r) + " (" #expr ")"); \
  } while (0)

#define HIP_CHECK(expr)                                                                             \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess)                                                                           \
      throw ClipErr(CLIPGPU_ERR_DEVICE, std::string("HIP error: ") + hipGetErrorString(_e) + " (" #expr \
                                            ")");                                                   \
  } while (0)

// MX-fp8 weight matrix (fp8 engines): e4m3 [N][K] + E8M0 scales [N][K/32] (gemm_mx.hip).
struct MxW {
  uint8_t* q = nullptr;
  uint8_t* s = nullptr;
};

struct LayerW {
  float *ln1_w, *ln1_b, *bqkv, *bo, *ln2_w, *ln2_b, *b1, *b2;
  // LayerNorm-folded engines (clipgpu_engine::lnf): wqkv / w1 hold W' = f16(W diag(gamma)), bqkv / b1
  // hold b + W beta, and these the column sums of W' (EPI_LNF)
  float *cs_qkv = nullptr, *cs_1 = nullptr;
  void *wqkv, *wo, *w1, *w2;  // 16-bit (fp8 engines: wo only)
  MxW mqkv, m1, m2;           // fp8 engines: QKV, c_fc, c_proj
};

// MAP attention-pool head of the SigLIP family (timm AttentionPoolLatent).
struct MapHeadW {
  float* q = nullptr;                 // [D] f32: latent . Wq^T + bq (the same for every image)
  void *wkv = nullptr, *wproj = nullptr, *w1 = nullptr, *w2 = nullptr;  // 16-bit [N][K]
  float *bkv = nullptr, *bproj = nullptr, *norm_w = nullptr, *norm_b = nullptr, *b1 = nullptr, *b2 = nullptr;
};

struct DevWeights {
  void* conv_w = nullptr;  // [D][Kpad] 16-bit (K = 3*P*P zero-padded to a multiple of 64)
  float* conv_b = nullptr; // SigLIP patch-embedding bias (nullptr for CLIP)
  MapHeadW map;
  float *cls = nullptr, *pos = nullptr, *lnpre_w = nullptr, *lnpre_b = nullptr;
  float* tok = nullptr;  // text token table [V][D] f32
  std::vector<LayerW> layers;
  float *lnpost_w = nullptr, *lnpost_b = nullptr;
  void* proj_t = nullptr;  // [E][D] 16-bit (transposed visual.proj / text_projection)
  float* proj_b = nullptr; // [E] text_projection.bias (SigLIP2 text; nullptr otherwise)
};

struct Replica {
  int device = 0;
  hipStream_t stream = nullptr;
  char* arena = nullptr;  // weights
  char* work = nullptr;   // activations
  DevWeights w;
  void* x = nullptr;      // [rows][D] residual stream: f32, or f16 (clipgpu_engine::x16)
  float* xs = nullptr;    // [rows + 256][2] (mean, rstd) of x's rows (LayerNorm-folded engines: ln_stats)
  void* h = nullptr;      // [rows][D] 16-bit (LN output / attention output); fp8 engines: LN output as e4m3
  uint8_t* hs = nullptr;   // fp8 engines: [rows][D/32] scales of the LN output in h
  uint8_t* bigs = nullptr; // fp8 engines: [rows][MLP/32] scales of the c_fc output (e4m3 in big)
  void* big = nullptr;    // [rows][max(3D, MLP)] 16-bit (qkv / MLP hidden)
  void* pooled = nullptr; // [B][D] 16-bit
  float* emb = nullptr;   // [B][E] f32 (pre-normalisation)
  float* out = nullptr;   // [B][E] f32
  void* in = nullptr;     // device input staging (pixels f32 / u8 / ids)
  void* pin_in = nullptr; // pinned host staging
  float* pin_out = nullptr;
  // Concurrent sub-batches ("lanes"): each lane runs the whole forward on a
  // contiguous slice of the batch on its own stream, so one lane's GEMM tail
  // rounds and memory-bound kernels overlap the other lane's GEMMs.
  hipStream_t lane[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t fork = nullptr, join[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t done[4] = {nullptr, nullptr, nullptr, nullptr};  // host path: chunk slot's D2H finished
  hipStream_t copy = nullptr, copy2 = nullptr;  // host path: every H2D, in chunk order; copy2: multi-round D2Hs
  hipEvent_t copied[4] = {nullptr, nullptr, nullptr, nullptr};  // host path: chunk slot's H2D finished
  // Host path, second buffer set (run_host_shard): a call of more than max_batch rows alternates
  // rounds between two sets of input / output staging, so round i + 1's host copy and H2D run under
  // round i's forward.  Allocated on the first such call (ensure_host_set2).
  void* in2 = nullptr;
  void* pin_in2 = nullptr;
  float* pin_out2 = nullptr;
  float* out2 = nullptr;  // set 1's device embedding rows
  hipEvent_t done2[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t copied2[4] = {nullptr, nullptr, nullptr, nullptr};
  // Decoded-image path (clipgpu_embed_images_rgb8): per slot, pinned staging and a device
  // arena of [descriptors | ints | raw RGB8 images], and the resize intermediate.  Grown
  // on demand (images have any size); reused across calls.
  struct ImageSlot {
    char* pin = nullptr;
    size_t pin_cap = 0;
    char* dev = nullptr;
    size_t dev_cap = 0;
    uint8_t* tmp = nullptr;
    size_t tmp_cap = 0;
  } islot[4];
  // Captured forwards (hipGraph), keyed by entry point, buffers and batch; owned here,
  // shared by the lane views.
  struct GraphCache* graphs = nullptr;
  hipEvent_t gin = nullptr, gout = nullptr;  // fork / join around a graph launched for a caller stream
  // RCCL communicator of this replica's rank (the one collective, an all-gather of
  // the embedding rows over xGMI): ncclCommInitAll over a multi-device handle's devices, or
  // ncclCommInitRank for one-process-per-GPU deployments (clipgpu_comm_init_rank).
  ncclComm_t comm = nullptr;
  hipEvent_t coll = nullptr;  // recorded behind this replica's last collective (destroy_comms waits for it)
};

// Replayable forwards: one hipGraphExec per (entry point, input / output buffers, batch,
// normalisation constants).  A forward is ~90 dependent launches per lane; replaying it
// as one graph removes the per-launch host cost and most inter-kernel dispatch gaps.
// Bounded: at kMax entries the least recently replayed one is destroyed, after every stream of
// the replica (the capture stream and the lane streams a host-path slot replays on) has drained,
// since any of them may still be running it.
struct GraphCache {
  struct Entry {
    std::vector<uint64_t> key;
    hipGraphExec_t exec;
    uint64_t last_use;
  };
  std::vector<Entry> entries;
  uint64_t clock = 0;
  static constexpr size_t kMax = 32;
  void clear() {
    for (auto& en : entries) (void)hipGraphExecDestroy(en.exec);
    entries.clear();
  }
};

}  // namespace clipgpu

namespace clipgpu {
// Live per-kernel-class timing with HIP events recorded on the launch stream
// (clipgpu_profile_*; bench.py's roofline.achieved).  Off by default.
enum ProfCat { PC_PATCH = 0, PC_STEM, PC_QKV, PC_ATTN, PC_OUT_PROJ, PC_LN, PC_C_FC, PC_C_PROJ, PC_HEAD, PC_TAIL, PC_N };
static const char* kProfNames[PC_N] = {"patch_embed", "stem_ln", "qkv", "attention", "out_proj",
                                       "layernorm", "c_fc", "c_proj", "head", "last_layer"};
struct Profiler {
  unsigned mask = 0;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  struct Rec { int cat; hipEvent_t a, b; hipStream_t st; };
  std::vector<Rec> pending;
  double total_ms[PC_N] = {0};
  long long count[PC_N] = {0};
  hipEvent_t get() {
    if (used == pool.size()) {
      hipEvent_t ev;
      if (hipEventCreate(&ev) != hipSuccess) return nullptr;
      pool.push_back(ev);
    }
    return pool[used++];
  }
};
}  // namespace clipgpu

struct clipgpu_engine {
  clipgpu::Profiler prof;
  // GEMM tile per trunk call site (clipgpu::GemmSite), autotuned at creation for
  // max_batch rows; batches under half of that use the shape heuristic.
  int tile[4] = {0, 0, 0, 0};
  int mxtile[4] = {0, 0, 0, 0};  // fp8 engines: MxTile of the MX sites (tile[] then holds the 16-bit tile
                                 // the site runs on layers outside mx_layers)
  int tile_patch = 0;  // vision: the patch-embedding GEMM (tuned with the trunk sites)
  int tuned_rows = 0;
  int lanes = 1;  // lane streams / host-path slots per device (clipgpu_options.lanes, default 2)
  // Concurrent sub-batches of a device-side forward: the tile table's choice, or `lanes` when
  // clipgpu_options.lanes pins it (full-batch GEMMs quantize better over the CUs than two
  // half-batch ones; the lanes overlap LayerNorm / attention with GEMMs).
  int dev_lanes = 1;
  bool lanes_pinned = false;
  bool graphs = true;  // replay forwards as hipGraphs (clipgpu_options.graphs = -1 disables)
  bool prune = true;   // last layer on the pooled rows only (clipgpu_options.prune_last = -1 disables; trunk)
  bool trim = true;    // host-ids text batches run on their first max(EOT)+1 tokens (options.trim_text = -1: off)
  // The residual stream x is stored in f16 (clipgpu_options.residual): its two read-modify-writes and
  // two LayerNorm reads per layer move half the bytes; every add into it and every LayerNorm statistic
  // stays f32.  bf16 / f16 engines of the CLIP family only (fp8 engines' MX residual epilogue and the
  // SigLIP MAP head take the f32 stream).
  bool x16 = false;
  // ln_1 / ln_2 folded into the QKV / c_fc GEMMs (clipgpu_options.ln_fold; f16 stream only): those
  // GEMMs read x (f16) with W' = W diag(gamma) (f16) and EPI_LNF; no LayerNorm launches in the trunk.
  bool lnf = false;

  int tuning = 0;  // clipgpu_options.tuning: 1 = timing tuner (+ whole-forward pass), 2 = per-site pass only
  // clipgpu_options.gemm_tiles / patch_tile pins (0 = the table's tile, -1 = the shape heuristic)
  int pin_tiles[4] = {0, 0, 0, 0};
  int pin_patch = 0;
  // fp8 engines: layer l runs its MX sites in MX-fp8 iff bit l is set (clipgpu_options.mx_layers; 0 =
  // every layer); the other layers run bf16 at every site
  uint64_t mx_layers = ~0ull;
  // Multi-device handles over distinct devices: the RCCL communicator is created on the first
  // gathered call (comm_pending), or at creation when clipgpu_options.communicator = 1.
  bool comm_pending = false;
  std::vector<int> comm_devs;
  bool force_bcast = false;  // test hook: gathered calls take the ragged (broadcast) branch
  // test hook (clipgpu_test_host_plan): the host path's chunk partition of max_batch (empty = host_chunks'
  // default)
  std::vector<int> host_part;
  // test hook (clipgpu_test_rgb8_resize_always): S x S decoded images also take the resize path
  bool rgb8_resize_always = false;
  clipgpu::TowerSpec spec;
  clipgpu::PreprocessCfg pre;
  clipgpu::DType dt = clipgpu::DT_BF16;
  // fp8 engine (CLIPGPU_DTYPE_FP8): QKV / c_fc / c_proj run as MX-fp8 GEMMs (e4m3 weights +
  // activations, E8M0 block scales, v_mfma_scale_f32_32x32x64_f8f6f4); attention, out_proj,
  // the stems and heads stay bf16.
  bool mx = false;
  // The MX sites of an fp8 engine (clipgpu_options.mx_sites, a subset of qkv / fc / proj; c_proj in MX
  // needs c_fc in MX, whose epilogue quantizes the hidden activations).  Default: all three.
  bool mx_site[4] = {false, false, false, false};  // indexed by GemmSite (GS_OUT stays bf16)
  int max_batch = 0;
  size_t in_bytes_per_row = 0;
  std::vector<clipgpu::Replica> reps;
  // Communicator geometry: comm_nranks ranks in all; replica i is rank comm_rank0 + i.
  int comm_nranks = 0, comm_rank0 = 0;
  std::mutex mu;  // one call per handle at a time (src/vision.rs:107 write lock)
};

namespace clipgpu {

namespace {

enum GemmSite { GS_QKV = 0, GS_OUT, GS_FC, GS_PROJ, GS_N };

// fp8 engines: does layer l run `site` as an MX-fp8 GEMM (the engine's MX sites, on the layers of
// clipgpu_options.mx_layers)?
inline bool mx_at(const clipgpu_engine& e, int l, int site) {
  return e.mx_site[site] && l >= 0 && l < 64 && ((e.mx_layers >> l) & 1ull);
}

inline size_t align256(size_t n) { return (n + 255) & ~size_t(255); }
inline int round64(int n) { return (n + 63) / 64 * 64; }
// GEMM K / N dims are multiples of 64: the MLP hidden width and the patch-embedding
// K = 3*P*P are zero-padded (exact: padded c_fc rows / bias are 0 and act(0) = 0 for
// every supported activation; padded conv columns multiply zero-filled pixels).
inline int mlp_pad(const TowerSpec& s) { return round64(s.mlp_width); }
inline int kpatch(const TowerSpec& s) { return 3 * s.patch_size * s.patch_size; }
inline int kpatch_pad(const TowerSpec& s) { return round64(kpatch(s)); }
// Elements per token row of the `big` scratch: QKV (3D), the MLP hidden width, and for
// the vision tower also the staged patch rows (G^2 rows of kpatch_pad per image, which
// the patch GEMM consumes before layer 0 writes QKV).
inline size_t big_wide(const TowerSpec& s) {
  size_t w = std::max((size_t)3 * s.width, (size_t)mlp_pad(s));
  if (s.tower == TOWER_VISION) {
    const size_t G = (size_t)s.image_size / s.patch_size, T = (size_t)s.tokens();
    w = std::max(w, (G * G * (size_t)kpatch_pad(s) + T - 1) / T);
  }
  return w;
}

bool file_exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

const HostTensor& need(const TensorMap& m, const std::string& k) {
  auto it = m.find(k);
  if (it == m.end()) throw ClipErr(CLIPGPU_ERR_CONFIG, "Configuration error: missing tensor " + k);
  return it->second;
}

// Bump allocator over a device arena.
struct Bump {
  char* base;
  size_t off = 0;
  size_t cap;
  void* take(size_t n) {
    void* p = base + off;
    off += align256(n);
    if (off > cap) throw ClipErr(CLIPGPU_ERR_DEVICE, "internal: arena overflow");
    return p;
  }
};

size_t weight_bytes(const TowerSpec& s, const TensorMap& m) {
  size_t total = 0;
  for (const ParamDesc& p : tower_params(s)) total += align256((size_t)need(m, p.name).numel() * 4);
  // zero padding of the MLP hidden width and of the patch K (16-bit matrices + f32 bias)
  const size_t mpad = (size_t)(mlp_pad(s) - s.mlp_width);
  total += (size_t)s.layers * (mpad * s.width * 4 + mpad * 4 + 1024);
  if (s.tower == TOWER_VISION) total += (size_t)(kpatch_pad(s) - kpatch(s)) * s.width * 2 + 256;
  if (s.family == FAMILY_SIGLIP) total += (mpad * s.width * 4 + mpad * 4) + (size_t)s.width * 4 + 4096;
  return total + 4096;
}

void upload_f32(const HostTensor& t, float* dst) {
  HIP_CHECK(copy_h2d(dst, t.data.data(), t.data.size() * 4));
}

void upload_16(DType dt, const float* src, size_t n, void* dst, float* staging, hipStream_t s) {
  HIP_CHECK(copy_h2d(staging, src, n * 4));
  HIP_CHECK(launch_cast_f32(dt, staging, dst, (long)n, s));
  HIP_CHECK(hipStreamSynchronize(s));
}

void upload_weights(clipgpu_engine& e, Replica& r, const TensorMap& m) {
  const TowerSpec& s = e.spec;
  const size_t bytes = weight_bytes(s, m);
  HIP_CHECK(hipMalloc(&r.arena, bytes));
  Bump a{r.arena, 0, bytes};
  const int D = s.width, E = s.embed_dim;
  size_t max16 = 0;
  for (const ParamDesc& p : tower_params(s)) max16 = std::max(max16, (size_t)need(m, p.name).numel());
  float* staging = nullptr;
  HIP_CHECK(hipMalloc(&staging, max16 * 4));
  std::vector<float*> extra_staging;
  auto staging_pad = [&](size_t n) {  // a padded matrix may exceed max16
    if (n <= max16) return staging;
    float* p = nullptr;
    HIP_CHECK(hipMalloc(&p, n * 4));
    extra_staging.push_back(p);
    return p;
  };
  auto f32 = [&](const std::string& k) {
    const HostTensor& t = need(m, k);
    float* p = (float*)a.take(t.data.size() * 4);
    upload_f32(t, p);
    return p;
  };
  auto w16 = [&](const std::string& k) {
    const HostTensor& t = need(m, k);
    void* p = a.take(t.data.size() * 2);
    upload_16(e.dt, t.data.data(), t.data.size(), p, staging, r.stream);
    return p;
  };
  // [R][C] -> zero-padded [Rp][Cp] (16-bit)
  auto w16_pad = [&](const std::string& k, int64_t Rp, int64_t Cp) {
    const HostTensor& t = need(m, k);
    const int64_t R = t.shape[0], C = t.numel() / t.shape[0];
    if (Rp == R && Cp == C) {
      void* p = a.take(t.data.size() * 2);
      upload_16(e.dt, t.data.data(), t.data.size(), p, staging, r.stream);
      return p;
    }
    std::vector<float> pad((size_t)(Rp * Cp), 0.f);
    for (int64_t i = 0; i < R; ++i)
      std::memcpy(&pad[(size_t)(i * Cp)], &t.data[(size_t)(i * C)], (size_t)C * 4);
    void* p = a.take(pad.size() * 2);
    upload_16(e.dt, pad.data(), pad.size(), p, staging_pad(pad.size()), r.stream);
    return p;
  };
  // [R][C] f32 -> zero-padded [Rp][Cp] MX-fp8 (quantized on the device)
  auto wmx_pad = [&](const std::string& k, int64_t Rp, int64_t Cp) {
    const HostTensor& t = need(m, k);
    const int64_t R = t.shape[0], C = t.numel() / t.shape[0];
    std::vector<float> pad;
    const float* src = t.data.data();
    if (Rp != R || Cp != C) {
      pad.assign((size_t)(Rp * Cp), 0.f);
      for (int64_t i = 0; i < R; ++i) std::memcpy(&pad[(size_t)(i * Cp)], &t.data[(size_t)(i * C)], (size_t)C * 4);
      src = pad.data();
    }
    float* stg = staging_pad((size_t)(Rp * Cp));
    HIP_CHECK(copy_h2d(stg, src, (size_t)(Rp * Cp) * 4));
    MxW w;
    w.q = (uint8_t*)a.take((size_t)(Rp * Cp));
    w.s = (uint8_t*)a.take((size_t)(Rp * Cp / 32));
    HIP_CHECK(launch_quant_rows(-1, stg, Cp, w.q, Cp, w.s, Cp / 32, (int)Rp, (int)Cp, r.stream));
    HIP_CHECK(hipStreamSynchronize(r.stream));
    return w;
  };
  auto f32_pad = [&](const std::string& k, int64_t n) {
    const HostTensor& t = need(m, k);
    std::vector<float> pad((size_t)n, 0.f);
    std::memcpy(pad.data(), t.data.data(), t.data.size() * 4);
    float* p = (float*)a.take(pad.size() * 4);
    HIP_CHECK(copy_h2d(p, pad.data(), pad.size() * 4));
    return p;
  };
  auto a_take_f32 = [&](const std::vector<float>& v) {
    float* p = (float*)a.take(v.size() * 4);
    HIP_CHECK(copy_h2d(p, v.data(), v.size() * 4));
    return p;
  };
  auto w16_transposed = [&](const std::string& k) {  // [D][E] -> [E][D]
    const HostTensor& t = need(m, k);
    const int64_t R = t.shape[0], C = t.shape[1];
    std::vector<float> tr((size_t)(R * C));
    for (int64_t i = 0; i < R; ++i)
      for (int64_t j = 0; j < C; ++j) tr[(size_t)(j * R + i)] = t.data[(size_t)(i * C + j)];
    void* p = a.take(tr.size() * 2);
    upload_16(e.dt, tr.data(), tr.size(), p, staging, r.stream);
    return p;
  };
  DevWeights& w = r.w;
  std::string pre;
  const bool siglip = s.tower == TOWER_VISION && s.family == FAMILY_SIGLIP;
  // parameter names of the two families (open_clip CLIP / timm ViT trunk)
  const char* n_ln1w = siglip ? "norm1.weight" : "ln_1.weight";
  const char* n_ln1b = siglip ? "norm1.bias" : "ln_1.bias";
  const char* n_qkvw = siglip ? "attn.qkv.weight" : "attn.in_proj_weight";
  const char* n_qkvb = siglip ? "attn.qkv.bias" : "attn.in_proj_bias";
  const char* n_ow = siglip ? "attn.proj.weight" : "attn.out_proj.weight";
  const char* n_ob = siglip ? "attn.proj.bias" : "attn.out_proj.bias";
  const char* n_ln2w = siglip ? "norm2.weight" : "ln_2.weight";
  const char* n_ln2b = siglip ? "norm2.bias" : "ln_2.bias";
  const char* n_fc1w = siglip ? "mlp.fc1.weight" : "mlp.c_fc.weight";
  const char* n_fc1b = siglip ? "mlp.fc1.bias" : "mlp.c_fc.bias";
  const char* n_fc2w = siglip ? "mlp.fc2.weight" : "mlp.c_proj.weight";
  const char* n_fc2b = siglip ? "mlp.fc2.bias" : "mlp.c_proj.bias";
  if (siglip) {
    const std::string t = "visual.trunk.";
    w.conv_w = w16_pad(t + "patch_embed.proj.weight", D, kpatch_pad(s));
    w.conv_b = f32(t + "patch_embed.proj.bias");
    w.pos = f32(t + "pos_embed");
    pre = t + "blocks.";
  } else if (s.tower == TOWER_VISION) {
    w.conv_w = w16_pad("visual.conv1.weight", D, kpatch_pad(s));
    w.cls = f32("visual.class_embedding");
    w.pos = f32("visual.positional_embedding");
    w.lnpre_w = f32("visual.ln_pre.weight");
    w.lnpre_b = f32("visual.ln_pre.bias");
    pre = "visual.transformer.resblocks.";
  } else {
    w.tok = f32("token_embedding.weight");
    w.pos = f32("positional_embedding");
    pre = "transformer.resblocks.";
  }
  // LayerNorm fold (clipgpu_engine::lnf) of the GEMM W [R][D] + b behind LayerNorm (gamma, beta):
  // W' = f16(W diag(gamma)) zero-padded to Rp rows, bias b + W beta (f64 sums, the f32 W), and the
  // column sums of W' as the kernel sees it (f16-rounded; f64 sums): LN(x) W^T + b =
  // rstd (x W'^T - mean cs) + b + W beta.
  auto fold_w = [&](const std::string& wk, const std::string& bk, const std::string& gk, const std::string& bek,
                    int64_t Rp, void*& wout, float*& bout, float*& csout) {
    const HostTensor& W = need(m, wk);
    const HostTensor& b = need(m, bk);
    const HostTensor& g = need(m, gk);
    const HostTensor& be = need(m, bek);
    const int64_t R = W.shape[0], C = W.numel() / W.shape[0];
    std::vector<float> wf((size_t)(Rp * C), 0.f), cs((size_t)Rp, 0.f), bp((size_t)Rp, 0.f);
    for (int64_t i = 0; i < R; ++i) {
      double sb = b.data[(size_t)i], sc = 0.0;
      for (int64_t k = 0; k < C; ++k) {
        const float wv = W.data[(size_t)(i * C + k)];
        const float wg = wv * g.data[(size_t)k];
        wf[(size_t)(i * C + k)] = wg;
        sc += (double)(float)(_Float16)wg;  // the device cast's rounding (to nearest even)
        sb += (double)wv * (double)be.data[(size_t)k];
      }
      cs[(size_t)i] = (float)sc;
      bp[(size_t)i] = (float)sb;
    }
    wout = a.take(wf.size() * 2);
    upload_16(DT_F16, wf.data(), wf.size(), wout, staging_pad(wf.size()), r.stream);
    bout = a_take_f32(bp);
    csout = a_take_f32(cs);
  };
  for (int l = 0; l < s.layers; ++l) {
    const std::string p = pre + std::to_string(l) + ".";
    LayerW L;
    L.ln1_w = f32(p + n_ln1w);
    L.ln1_b = f32(p + n_ln1b);
    L.wqkv = L.w1 = L.w2 = nullptr;
    if (e.lnf) fold_w(p + n_qkvw, p + n_qkvb, p + n_ln1w, p + n_ln1b, 3 * D, L.wqkv, L.bqkv, L.cs_qkv);
    else if (mx_at(e, l, GS_QKV)) L.mqkv = wmx_pad(p + n_qkvw, 3 * D, D);
    else L.wqkv = w16(p + n_qkvw);
    if (e.lnf) fold_w(p + n_fc1w, p + n_fc1b, p + n_ln2w, p + n_ln2b, mlp_pad(s), L.w1, L.b1, L.cs_1);
    else if (mx_at(e, l, GS_FC)) L.m1 = wmx_pad(p + n_fc1w, mlp_pad(s), D);
    else L.w1 = w16_pad(p + n_fc1w, mlp_pad(s), D);
    if (mx_at(e, l, GS_PROJ)) L.m2 = wmx_pad(p + n_fc2w, D, mlp_pad(s));
    else L.w2 = w16_pad(p + n_fc2w, D, mlp_pad(s));
    if (!e.lnf) L.bqkv = f32(p + n_qkvb);
    L.wo = w16(p + n_ow);
    L.bo = f32(p + n_ob);
    L.ln2_w = f32(p + n_ln2w);
    L.ln2_b = f32(p + n_ln2b);
    if (!e.lnf) L.b1 = f32_pad(p + n_fc1b, mlp_pad(s));
    L.b2 = f32(p + n_fc2b);
    w.layers.push_back(L);
  }
  if (siglip) {
    const std::string t = "visual.trunk.", a = "visual.trunk.attn_pool.";
    w.lnpost_w = f32(t + "norm.weight");  // final norm, before the attention pool
    w.lnpost_b = f32(t + "norm.bias");
    {  // q = latent . Wq^T + bq, shared by every image (f64 accumulation)
      const HostTensor& lat = need(m, a + "latent");
      const HostTensor& wq = need(m, a + "q.weight");
      const HostTensor& bq = need(m, a + "q.bias");
      std::vector<float> q((size_t)D);
      for (int j = 0; j < D; ++j) {
        double acc = bq.data[(size_t)j];
        for (int i = 0; i < D; ++i) acc += (double)lat.data[(size_t)i] * wq.data[(size_t)j * D + i];
        q[(size_t)j] = (float)acc;
      }
      w.map.q = (float*)a_take_f32(q);
    }
    w.map.wkv = w16(a + "kv.weight");
    w.map.bkv = f32(a + "kv.bias");
    w.map.wproj = w16(a + "proj.weight");
    w.map.bproj = f32(a + "proj.bias");
    w.map.norm_w = f32(a + "norm.weight");
    w.map.norm_b = f32(a + "norm.bias");
    w.map.w1 = w16_pad(a + "mlp.fc1.weight", mlp_pad(s), D);
    w.map.b1 = f32_pad(a + "mlp.fc1.bias", mlp_pad(s));
    w.map.w2 = w16_pad(a + "mlp.fc2.weight", D, mlp_pad(s));
    w.map.b2 = f32(a + "mlp.fc2.bias");
  } else if (s.tower == TOWER_VISION) {
    w.lnpost_w = f32("visual.ln_post.weight");
    w.lnpost_b = f32("visual.ln_post.bias");
    w.proj_t = w16_transposed("visual.proj");
  } else {
    w.lnpost_w = f32("ln_final.weight");
    w.lnpost_b = f32("ln_final.bias");
    if (s.proj_bias) {  // nn.Linear: weight already [E][D]
      w.proj_t = w16("text_projection.weight");
      w.proj_b = f32("text_projection.bias");
    } else {
      w.proj_t = w16_transposed("text_projection");
    }
  }
  (void)D;
  (void)E;
  HIP_CHECK(hipFree(staging));
  for (float* p : extra_staging) HIP_CHECK(hipFree(p));
}

void alloc_workspace(clipgpu_engine& e, Replica& r) {
  const TowerSpec& s = e.spec;
  // lanes x ceil(max_batch / lanes) rows: every host-path slot (run_host_shard) is whole
  const size_t B = (size_t)((e.max_batch + e.lanes - 1) / e.lanes * e.lanes);
  const size_t rows = B * (size_t)s.tokens(), D = s.width;
  const size_t wide = big_wide(s);
  const size_t E = s.embed_dim;
  const size_t MLP = (size_t)mlp_pad(s);
  const size_t sizes[] = {rows * D * 4, rows * D * 2, rows * wide * 2, B * D * 2, B * E * 4, B * E * 4,
                          B * e.in_bytes_per_row, e.mx ? rows * D / 32 : 0, e.mx ? rows * MLP / 32 : 0,
                          (rows + 256) * 8};
  size_t total = 0;
  for (size_t z : sizes) total += align256(z);
  HIP_CHECK(hipMalloc(&r.work, total));
  HIP_CHECK(hipMemset(r.work, 0, total));
  Bump a{r.work, 0, total};
  r.x = a.take(sizes[0]);  // f32 capacity (an f16 stream uses the first half)
  r.h = a.take(sizes[1]);
  r.big = a.take(sizes[2]);
  r.pooled = a.take(sizes[3]);
  r.emb = (float*)a.take(sizes[4]);
  r.out = (float*)a.take(sizes[5]);
  r.in = a.take(sizes[6]);
  r.hs = e.mx ? (uint8_t*)a.take(sizes[7]) : nullptr;
  r.bigs = e.mx ? (uint8_t*)a.take(sizes[8]) : nullptr;
  r.xs = (float*)a.take(sizes[9]);
  for (int i = 0; i < e.lanes; ++i) {
    HIP_CHECK(hipStreamCreateWithFlags(&r.lane[i], hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&r.join[i], hipEventDisableTiming));
  }
  for (int i = 0; i < 4; ++i) {  // host-path chunks: up to 4 (host_chunks), independent of the lanes
    HIP_CHECK(hipEventCreateWithFlags(&r.done[i], hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&r.copied[i], hipEventDisableTiming));
  }
  HIP_CHECK(hipStreamCreateWithFlags(&r.copy, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&r.copy2, hipStreamNonBlocking));
  HIP_CHECK(hipEventCreateWithFlags(&r.fork, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&r.gin, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&r.gout, hipEventDisableTiming));
  r.graphs = new GraphCache();
  HIP_CHECK(hipHostMalloc(&r.pin_in, B * e.in_bytes_per_row, hipHostMallocDefault));
  HIP_CHECK(hipHostMalloc((void**)&r.pin_out, B * E * 4, hipHostMallocDefault));
}

void check(hipError_t err, const char* what) {
  if (err != hipSuccess) {
    (void)hipGetLastError();  // reported here; do not let the next call's launch check see it again
    throw ClipErr(CLIPGPU_ERR_DEVICE, std::string("HIP error in ") + what + ": " + hipGetErrorString(err));
  }
}

// Times the launches of one scope when its category is enabled.  gemm = true (a single
// launch_gemm inside): the events are handed to the GEMM launcher, which stamps the kernel's
// own start and end (hipExtLaunchKernelGGL); otherwise [start, stop] are recorded around the
// scope's launches on the stream (which also counts their dispatch gaps).
struct ProfScope {
  Profiler* p;
  int cat;
  hipStream_t st;
  bool gemm;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(const clipgpu_engine& e, int c, hipStream_t s, bool gemm_scope = false)
      : p(const_cast<Profiler*>(&e.prof)), cat(c), st(s), gemm(gemm_scope) {
    if (p->mask & (1u << cat)) {
      a = p->get();
      b = a ? p->get() : nullptr;
      if (!b) {
        a = nullptr;
      } else if (gemm) {
        g_gemm_events.start = a;
        g_gemm_events.stop = b;
      } else {
        (void)hipEventRecord(a, st);
      }
    }
  }
  ~ProfScope() {
    if (!a) return;
    if (gemm) g_gemm_events = GemmLaunchEvents();  // consumed by the launch (or disarm on error)
    else (void)hipEventRecord(b, st);
    p->pending.push_back({cat, a, b, st});
  }
};

GemmParams rows_gemm(const void* A, long lda, const void* W, const float* bias, void* out, long ldo, int M, int N,
                     int K) {
  GemmParams g{};
  g.A = A;
  g.lda = lda;
  g.W = W;
  g.ldw = K;
  g.bias = bias;
  g.out = out;
  g.ldo = ldo;
  g.M = M;
  g.N = N;
  g.K = K;
  return g;
}

// The residual stream's element size and row offsets (f32, or f16: clipgpu_engine::x16).
inline size_t xbytes(const clipgpu_engine& e) { return e.x16 ? 2 : 4; }
inline void* xrows(const clipgpu_engine& e, void* x, size_t rows) {
  return (char*)x + rows * (size_t)e.spec.width * xbytes(e);
}

// clipgpu_options.residual = 0: the residual stream's default storage
constexpr int kResidualDefault = CLIPGPU_RESIDUAL_F16;

int site_epi(const clipgpu_engine& e, int site) {
  if (site == GS_OUT || site == GS_PROJ) return EPI_RESID;
  return e.lnf ? EPI_LNF : EPI_STORE16;  // QKV / c_fc behind the folded LayerNorm
}

// Tile order per trunk site (GemmParams.group: row panels per group, 0 = the kernels' 8).  qkv and
// c_proj walk N first (group 1): their W (3 D x D, D x MLP) is small beside A, so each XCD reads an A
// row panel once and all of W, instead of every panel from two XCDs: c_proj's fetched bytes at the
// ViT-B/32 lane shape drop from 1.96x to ~1.4x its compulsory bytes.  Speed
// only: the order never changes a tile's sums.  (CLIPGPU_SITE_GROUPS=0 builds the uniform order for
// A/B runs.)
#ifndef CLIPGPU_SITE_GROUPS
#define CLIPGPU_SITE_GROUPS 1
#endif
constexpr int kSiteGroup[4] = {CLIPGPU_SITE_GROUPS ? 1 : 0, 0, 0, CLIPGPU_SITE_GROUPS ? 1 : 0};

GemmParams site_gemm(const clipgpu_engine& e, const Replica& r, const LayerW& L, int site, int rows) {
  const int D = e.spec.width, MLP = mlp_pad(e.spec);
  GemmParams g;
  // (LayerNorm-folded engines: QKV and c_fc read the residual stream x itself, EPI_LNF)
  const void* ln_in = e.lnf ? r.x : r.h;
  switch (site) {
    case GS_QKV: g = rows_gemm(ln_in, D, L.wqkv, L.bqkv, r.big, 3 * D, rows, 3 * D, D); break;
    case GS_OUT: g = rows_gemm(r.h, D, L.wo, L.bo, r.x, D, rows, D, D); break;
    case GS_FC: g = rows_gemm(ln_in, D, L.w1, L.b1, r.big, MLP, rows, MLP, D); break;
    default: g = rows_gemm(r.big, MLP, L.w2, L.b2, r.x, D, rows, D, MLP); break;
  }
  if (e.lnf && (site == GS_QKV || site == GS_FC)) {
    g.cs = site == GS_QKV ? L.cs_qkv : L.cs_1;
    g.rowstats = r.xs;
  }
  g.group = kSiteGroup[site];
  g.x16 = e.x16 ? 1 : 0;
  // the younger half of 8-wave blocks at priority 1: vision +0.75 %, text -0.5 % (gemm.hip)
  g.prio = e.spec.tower == TOWER_VISION ? 1 : 0;
  return g;
}

// fp8 engines: the MX-fp8 GEMM of a trunk site (QKV: LN e4m3 -> 16-bit qkv; c_fc: LN e4m3 ->
// act -> e4m3 hidden in `big` + scales; c_proj: e4m3 hidden -> residual stream).
// c_fc quantizes its output (EPI_STOREQ) only when the layer's c_proj consumes MX; else it stores 16-bit.
int site_epi_mx(const clipgpu_engine& e, int l, int site) {
  return site == GS_PROJ ? EPI_RESID : (site == GS_FC && mx_at(e, l, GS_PROJ) ? EPI_STOREQ : EPI_STORE16);
}
// LN output feeding an MX GEMM (layer l's consumer site) is written as MX-fp8 (scales in hs), else 16-bit.
inline uint8_t* ln_q(const clipgpu_engine& e, int l, int consumer_site, uint8_t* hs) {
  return mx_at(e, l, consumer_site) ? hs : nullptr;
}

MxGemmParams site_gemm_mx(const clipgpu_engine& e, const Replica& r, const LayerW& L, int site, int rows) {
  const int D = e.spec.width, MLP = mlp_pad(e.spec);
  MxGemmParams g{};
  g.M = rows;
  if (site == GS_PROJ) {
    g.A = (const uint8_t*)r.big; g.lda = MLP; g.As = r.bigs; g.ldas = MLP / 32;
    g.W = L.m2.q; g.ldw = MLP; g.Ws = L.m2.s; g.ldws = MLP / 32;
    g.bias = L.b2; g.out = r.x; g.ldo = D; g.N = D; g.K = MLP;
    g.x16 = e.x16 ? 1 : 0;
    return g;
  }
  g.A = (const uint8_t*)r.h; g.lda = D; g.As = r.hs; g.ldas = D / 32;
  g.K = D;
  if (site == GS_QKV) {
    g.W = L.mqkv.q; g.ldw = D; g.Ws = L.mqkv.s; g.ldws = D / 32;
    g.bias = L.bqkv; g.out = r.big; g.ldo = 3 * D; g.N = 3 * D;
  } else {  // GS_FC
    g.W = L.m1.q; g.ldw = D; g.Ws = L.m1.s; g.ldws = D / 32;
    g.bias = L.b1; g.out = r.big; g.ldo = MLP; g.outs = r.bigs; g.ldos = MLP / 32; g.N = MLP;
  }
  return g;
}

#ifdef CLIPGPU_ABLATE
// Diagnostic build only (make variant VNAME=ablate VDEFS=-DCLIPGPU_ABLATE; tools/ablate.py): skips
// trunk ops so that each op's marginal share of the concurrent-lane step can be measured (the
// numbers are garbage).  Bits: 0 LayerNorm, 1 attention, 2 out_proj, 3 qkv, 4 c_fc, 5 c_proj.
// The product library has no such switch.
static unsigned g_ablate = 0;
#define ABLATED(bit) ((g_ablate >> (bit)) & 1u)
extern "C" int clipgpu_test_ablate(unsigned mask) {
  g_ablate = mask;
  return 0;
}
#else
#define ABLATED(bit) false
#endif

// Residual rows the head pools from: x at token pos(b) of each sequence (tokens = T), or the
// compact [B][D] rows the pruned last layer leaves (tokens = 1, pos 0).
struct PoolSrc {
  const void* x;  // the residual stream's type (clipgpu_engine::x16)
  int tokens;
  const int64_t* ids;
};

// Last-layer pruning.  The CLIP heads read one token per sequence (CLS, or the EOT argmax
// for text), and after the last layer's attention every op is row-local (out_proj, ln_2,
// c_fc, c_proj), so that layer's tail runs on the pooled rows only: attention still reads
// every token's K/V, then the pooled token's residual row and attention output are gathered
// to a compact [B][D] pair and out_proj .. c_proj run at M = B.  Each kept row goes through
// the same kernels with the same K-ordered sums, so the embeddings are bit-identical to the
// full last layer (test_last_layer_pruning_is_bit_exact).  Off with clipgpu_options.prune_last = -1;
// not for the SigLIP MAP head (pools every token).
// The compact pair lives in the tail of `big`, past the M = B MLP hidden.
inline size_t prune_off_x(const TowerSpec& s, int B) { return align256((size_t)B * mlp_pad(s) * 2); }
inline size_t prune_off_h(const TowerSpec& s, int B) {
  return prune_off_x(s, B) + align256((size_t)B * s.width * 4);
}
inline size_t prune_off_xs(const TowerSpec& s, int B) {  // the compact rows' statistics (ln_fold)
  return prune_off_h(s, B) + align256((size_t)B * s.width * 2);
}
inline bool prune_last(const clipgpu_engine& e, int B, int T) {
  const TowerSpec& s = e.spec;
  return e.prune && s.family != FAMILY_SIGLIP && s.layers > 0 &&
         prune_off_xs(s, B) + ((size_t)B + 256) * 8 <= (size_t)B * T * big_wide(s) * 2;
}

// The transformer trunk shared by both towers: L x [LN1 -> QKV -> MHA -> out+res ->
// LN2 -> fc1+act -> fc2+res], with h already holding ln_1(x) of layer 0.  ids: the text
// tower's token ids (pooled-token choice when the last layer is pruned), nullptr for CLS.
// T: tokens per sequence (the text tower's trimmed length, else the tower's own).
PoolSrc trunk(const clipgpu_engine& e, const Replica& r, int B, int causal, const int64_t* ids, hipStream_t st,
              int T, int pool_pos = 0) {
  const TowerSpec& s = e.spec;
  const int D = s.width;
  const bool prune = prune_last(e, B, T);
  for (int l = 0; l < s.layers; ++l) {
    const LayerW& L = r.w.layers[l];
    const bool compact = prune && l + 1 == s.layers;
    Replica c = r;  // the buffers the tail of this layer runs on
    int rows = B * T;
    auto gemm = [&](int site, int cat, const char* what) {
      if (ABLATED(site == GS_QKV ? 3 : site == GS_OUT ? 2 : site == GS_FC ? 4 : 5)) return;
      ProfScope ps(e, rows == B * T ? cat : PC_TAIL, st, /*gemm=*/true);
      const bool tuned = 2 * rows > e.tuned_rows;
      if (mx_at(e, l, site)) {
        MxGemmParams g = site_gemm_mx(e, c, L, site, rows);
        g.tile = tuned ? e.mxtile[site] : MX_TILE_AUTO;
        check(launch_gemm_mx(e.dt, site_epi_mx(e, l, site), site == GS_FC ? s.act : ACT_NONE, g, st), what);
        return;
      }
      GemmParams g = site_gemm(e, c, L, site, rows);
      g.tile = tuned ? e.tile[site] : TILE_AUTO;
      check(launch_gemm(e.dt, A_ROWS, site_epi(e, site), site == GS_FC ? s.act : ACT_NONE, g, st), what);
    };
    gemm(GS_QKV, PC_QKV, "qkv gemm");
    if (!ABLATED(1)) { ProfScope ps(e, PC_ATTN, st);
      check(launch_attention(e.dt, r.big, r.h, B, T, s.heads, D, causal, st), "attention"); }
    if (compact) {  // pooled rows only from here on (QKV in `big` is dead after attention)
      c.x = (char*)r.big + prune_off_x(s, B);
      c.h = (char*)r.big + prune_off_h(s, B);
      c.xs = (float*)((char*)r.big + prune_off_xs(s, B));
      rows = B;
      ProfScope ps(e, PC_TAIL, st);
      // ids == nullptr: position pool_pos of every sequence (CLS 0, SigLIP2 text T - 1)
      check(launch_gather_pooled(xrows(e, r.x, pool_pos), e.x16, (char*)r.h + (size_t)pool_pos * D * 2, ids, T, c.x, c.h,
                                 B, D, st),
            "gather pooled rows");
    }
    gemm(GS_OUT, PC_OUT_PROJ, "out_proj gemm");
    if (!ABLATED(0)) {
      ProfScope ps(e, compact ? PC_TAIL : PC_LN, st);
      if (e.lnf)  // (folded into c_fc: its rows' statistics only)
        check(launch_ln_stats(c.x, 1, s.ln_eps, c.xs, rows, D, st), "ln_2 statistics");
      else
        check(launch_ln_rows(e.dt, c.x, e.x16, L.ln2_w, L.ln2_b, s.ln_eps, c.h, rows, D, st, ln_q(e, l, GS_FC, c.hs)),
              "ln_2");
    }
    gemm(GS_FC, PC_C_FC, "c_fc gemm");
    gemm(GS_PROJ, PC_C_PROJ, "c_proj gemm");
    if (l + 1 < s.layers && !ABLATED(0)) {
      ProfScope ps(e, PC_LN, st);
      if (e.lnf)  // (folded into the next QKV: its rows' statistics only)
        check(launch_ln_stats(r.x, 1, s.ln_eps, r.xs, rows, D, st), "ln_1 statistics");
      else
        check(launch_ln_rows(e.dt, r.x, e.x16, r.w.layers[l + 1].ln1_w, r.w.layers[l + 1].ln1_b, s.ln_eps, r.h, rows,
                             D, st, ln_q(e, l + 1, GS_QKV, r.hs)),
              "ln_1");
    }
    if (compact) return PoolSrc{c.x, 1, nullptr};
  }
  return PoolSrc{xrows(e, r.x, pool_pos), T, ids};
}

// The committed MI355X tile table (default; clipgpu_options.tuning = 0).  A trunk site's tile is
// a function of its GEMM shape at the rows one lane runs at max_batch, so an engine's kernels --
// and the profiles and PMC records taken of them -- are the same on every box and every run.  The
// entries are the timing tuner's (below) majority choice over repeated runs on MI355X
// (tools/tile_table.py, profiles/r03_v13_tile_table.jsonl); the tile choice never changes the output
// bits (every tile computes the same K-ordered sums, test_gemm_tile_choice_is_bit_exact).
//   qkv / c_fc (N = 3D / MLP wide, K = D): 256x256 with the half-tile last round (tile 18, which
//     falls back to plain 256x256 RS where the half round does not apply);
//   out_proj / c_proj (N = D, + residual): 160x128 8-wave RS (tile 17), two blocks per CU; except
//     the wide, K-long c_proj of ViT-H/14 (N >= 1280, K >= 5120): 192x256 8-wave (tile 13), 681-685
//     vs 725-740 us at 46720 x 1280 x 5120 in two interleaved A/B sessions
//     (profiles/r03_v2_gemm_ab_pp.txt, r03_v7_tile_256x128_half_ab.txt); at every other N = D shape
//     of the BASELINE models tile 17 is the fastest or within 1 %;
//   rows < 2048 (small max_batch): the shape heuristic (TILE_AUTO; skinny kernel <= 256 rows).
// `rows` is one lane's rows at max_batch; the lane count is table_lanes' (below), and the two-lane
// ViT-B/32 regime overrides out_proj / c_fc / c_proj / patch in table_tiles.
int table_tile(int site, int rows, int N, int K) {
  if (rows < 2048) return TILE_AUTO;
  switch (site) {
    case GS_QKV: return TILE_256x256_HALF;
    case GS_FC: return TILE_256x256_HALF;
    default: return N >= 1280 && K >= 5120 ? TILE_192x256_W8 : TILE_160x128_W8_RS;
  }
}

// Device lanes of the committed table.  A large-batch text tower (>= 32768 token rows: configs[2]'s
// 1024 x 77) takes two lanes: its LayerNorms and causal attention are a larger
// share of the layer than in the vision trunk (0.7 + 0.7 ms of 9.3 ms at one lane) and overlap the
// other lane's GEMMs, while 39424-row lanes still fill the 256x256 / 160x128 rounds (round 2's
// two-lane text leg: 117k seq/s; round 3's one-lane table: 110k; profiles/r03_v12_text_lanes_ab.txt).
// Round 4: a vision batch of 8192..32767 token rows (ViT-B/32 at 256 images: 12800) takes two
// lanes too, with out_proj, c_fc, c_proj and the patch GEMM off the 8-wave 160x128 tile (table_tiles
// below: c_fc on the 4-wave 160x128 RS tile, two blocks per CU, one from each lane).  Same-box A/Bs (tools/bench_variants.sh,
// profiles/r04_lanes_ab.jsonl): one lane on the 8-wave table tiles 79.8-80.3k img/s; two lanes on the
// same tiles 81.3k; two lanes with these 82.6-84.2k (qkv on 256x256 plain, RS or half-tile within
// 0.5 %; c_fc on 256x256 at two lanes loses 2 %).  The round-1 tree -- two lanes of 160x128 tiles
// -- ran 83.4k on the same box as this tree's one-lane table's 79.8k (profiles/r04_ab_trees.jsonl):
// round 3's move to one lane was the 80.9k of BENCH_r03.
constexpr long kVisionTwoLaneRows[2] = {8192, 32768};
bool vision_two_lanes(const clipgpu_engine& e) {
  const long rows = (long)e.max_batch * e.spec.tokens();
  return e.spec.tower == TOWER_VISION && rows >= kVisionTwoLaneRows[0] && rows < kVisionTwoLaneRows[1];
}
// Larger vision batches take two lanes on their one-lane tiles: DFN5B ViT-H/14-378 at 64 images
// (46720 rows) 862 -> 886 img/s, SO400M-16-SigLIP2-384 at 128 (73728 rows) 1545 -> 1545
// (tools/bench_models.py lanesab, profiles/r04_large_model_lanes_ab.jsonl, two rounds each).
int table_lanes(const clipgpu_engine& e) {
  const long rows = (long)e.max_batch * e.spec.tokens();
  if (e.spec.tower == TOWER_VISION) return rows >= kVisionTwoLaneRows[0] ? 2 : 1;
  return e.spec.tower == TOWER_TEXT && rows >= 32768 ? 2 : 1;
}

void table_tiles(clipgpu_engine& e) {
  if (!e.lanes_pinned) e.dev_lanes = table_lanes(e);
  const int rows = (e.max_batch + e.dev_lanes - 1) / e.dev_lanes * e.spec.tokens();
  e.tuned_rows = rows;
  const int D = e.spec.width, MLP = mlp_pad(e.spec);
  const int shape[GS_N][2] = {{3 * D, D}, {D, D}, {MLP, D}, {D, MLP}};
  for (int site = 0; site < GS_N; ++site) {
    e.tile[site] = table_tile(site, rows, shape[site][0], shape[site][1]);
    e.mxtile[site] = MX_TILE_AUTO;
  }
  // Large text batches: c_proj (N = 512, K = 2048) on the 4-wave 160x128 RS tile, two blocks per CU
  // beside the other lane's work: 113.2-113.7k -> 116.6-116.8k seq/s in a same-box A/B against
  // the 8-wave tile 17 (profiles/r03_v13_text_tiles_ab.txt; the tuner's pick was 15 as well)
  // (measured for the two-lane regime only, so tied to it)
  if (e.spec.tower == TOWER_TEXT && e.dev_lanes == 2 && rows >= 16384) e.tile[GS_PROJ] = TILE_160x128_RS;
  // the patch-embedding GEMM has the c_proj shape class (N = D, K = 3 P^2 padded)
  const int G = e.spec.grid();
  const int prow = e.spec.tower == TOWER_VISION ? rows / e.spec.tokens() * G * G : 0;
  e.tile_patch = prow >= 2048 ? TILE_160x128_W8_RS : TILE_AUTO;
  // the two-lane vision regime (table_lanes): qkv, c_fc, c_proj and the patch GEMM (c_proj's shape class)
  // on the 4-wave 160x128 RS tile (two blocks per CU), out_proj on the 8-wave 224x192 tile (one round of
  // 116 tiles per 6400-row lane).  qkv moved off the 256x256 half tile in round 6: the same 26 us alone,
  // 94.2k vs 92.9k img/s in the forward (profiles/r06_qkv_tile_ab.txt).  Round 4 put c_proj on 224x192 too (+0.4-0.9 %, f32 stream,
  // profiles/r04_residual26_two_lanes_ab.jsonl); with the f16 stream and the round-6 DMA issue,
  // c_proj alone takes 41.4 us on 160x128 against 57.1 us on 224x192 and the step is as fast or faster
  // (93.1k vs 92.3k img/s, profiles/r06_residual_tiles_ab.txt); c_fc on 224x192 loses 3 %
  if (vision_two_lanes(e) && e.dev_lanes == 2 && rows >= 2048) {
    e.tile[GS_QKV] = e.tile[GS_FC] = e.tile[GS_PROJ] = TILE_160x128_RS;
    e.tile[GS_OUT] = TILE_224x192_W8;
    if (prow >= 2048) e.tile_patch = TILE_160x128_RS;
    if (e.mx) {  // fp8 engines: the timing tuner's picks in this regime, 105.0k vs 102.6k img/s over the MX
                 // shape heuristic (profiles/r06_fp8_tiles_probe.jsonl)
      e.mxtile[GS_QKV] = MX_TILE_256x128;
      e.mxtile[GS_FC] = e.mxtile[GS_PROJ] = MX_TILE_128x128;
      e.tile[GS_OUT] = TILE_160x128_RS;
    }
  }
}

// clipgpu_options.gemm_tiles / patch_tile pins over the table's (or the tuner's) choice: a GemmTile
// id, or -1 = the shape heuristic (TILE_AUTO).  Validated at creation (built tiles only).
void apply_tile_pins(clipgpu_engine& e) {
  for (int i = 0; i < GS_N; ++i)
    if (e.pin_tiles[i]) e.tile[i] = e.pin_tiles[i] < 0 ? TILE_AUTO : e.pin_tiles[i];
  if (e.pin_patch) e.tile_patch = e.pin_patch < 0 ? TILE_AUTO : e.pin_patch;
}
bool tiles_pinned(const clipgpu_engine& e) {
  bool any = e.pin_patch != 0;
  for (int t : e.pin_tiles) any = any || t != 0;
  return any;
}

// The tiles both timing passes choose from (the per-site autotune and tune_forward's coordinate
// descent): every tile the library builds (kGemmTiles).
const auto& kTuneCands = kGemmTiles;

// Timing tuner (clipgpu_options.tuning = 1 / 2; tools/tile_table.py uses it to regenerate the table):
// times each candidate tile on every trunk GEMM site at max_batch rows (workspace contents are
// scratch at this point) and keeps the fastest.  Tile choice changes speed only: every tile computes
// the same sums in the same K order.
void autotune_tiles(clipgpu_engine& e, Replica& r) {
  // tuned for the rows one lane runs at max_batch
  const int rows = (e.max_batch + e.dev_lanes - 1) / e.dev_lanes * e.spec.tokens();
  e.tuned_rows = rows;
  const auto& cands = kTuneCands;
  hipEvent_t a, b;
  HIP_CHECK(hipEventCreate(&a));
  HIP_CHECK(hipEventCreate(&b));
  auto tune = [&](GemmParams g, int epi, int act) {
    float best = 1e30f;
    int best_tile = TILE_AUTO;
    for (int t : cands) {
      g.tile = t;
      check(launch_gemm(e.dt, A_ROWS, epi, act, g, r.stream), "autotune gemm");
      HIP_CHECK(hipEventRecord(a, r.stream));
      const int iters = 4;
      for (int i = 0; i < iters; ++i) check(launch_gemm(e.dt, A_ROWS, epi, act, g, r.stream), "autotune gemm");
      HIP_CHECK(hipEventRecord(b, r.stream));
      HIP_CHECK(hipEventSynchronize(b));
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) {
        best = ms;
        best_tile = t;
      }
    }
    return best_tile;
  };
  const LayerW& L = r.w.layers[0];
  for (int site = 0; site < GS_N; ++site) {
    if (mx_at(e, 0, site)) {  // MX sites: the built MX tiles (same timing loop)
      MxGemmParams g = site_gemm_mx(e, r, L, site, rows);
      const int epi = site_epi_mx(e, 0, site), act = site == GS_FC ? e.spec.act : ACT_NONE;
      float best = 1e30f;
      for (int t : {MX_TILE_256x128, MX_TILE_128x128}) {
        g.tile = t;
        check(launch_gemm_mx(e.dt, epi, act, g, r.stream), "autotune mx gemm");
        HIP_CHECK(hipEventRecord(a, r.stream));
        for (int i = 0; i < 4; ++i) check(launch_gemm_mx(e.dt, epi, act, g, r.stream), "autotune mx gemm");
        HIP_CHECK(hipEventRecord(b, r.stream));
        HIP_CHECK(hipEventSynchronize(b));
        float ms = 0.f;
        HIP_CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) {
          best = ms;
          e.mxtile[site] = t;
        }
      }
    }
    if (e.mx && (e.mx_layers & 1ull) && e.mx_site[site]) {
      // a 16-bit GEMM runs at this site only on layers outside mx_layers: the table's tile there
      const int D = e.spec.width, MLP = mlp_pad(e.spec);
      const int shape[GS_N][2] = {{3 * D, D}, {D, D}, {MLP, D}, {D, MLP}};
      e.tile[site] = table_tile(site, rows, shape[site][0], shape[site][1]);
      continue;
    }
    e.tile[site] = tune(site_gemm(e, r, L, site, rows), site_epi(e, site), site == GS_FC ? e.spec.act : ACT_NONE);
  }
  if (e.spec.tower == TOWER_VISION) {
    const TowerSpec& s = e.spec;
    const int G = s.grid(), Kp = kpatch_pad(s), lane_b = rows / s.tokens();
    GemmParams g = rows_gemm(r.big, Kp, r.w.conv_w, r.w.conv_b, r.x, s.width, lane_b * G * G, s.width, Kp);
    g.G = G;
    g.pos = r.w.pos;
    g.cls = s.cls() ? 1 : 0;
    g.x16 = e.x16 ? 1 : 0;
    e.tile_patch = tune(g, EPI_PATCH, ACT_NONE);
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
}

void head(const clipgpu_engine& e, const Replica& r, int B, const PoolSrc& src, float* d_out, hipStream_t st) {
  const TowerSpec& s = e.spec;
  const int D = s.width, E = s.embed_dim;
  ProfScope ps(e, PC_HEAD, st);
  check(launch_pool_ln(e.dt, src.x, e.x16, src.ids, src.tokens, r.w.lnpost_w, r.w.lnpost_b, s.ln_eps, r.pooled, B, D,
                       st),
        "pool+ln");
  check(launch_gemm(e.dt, A_ROWS, EPI_STORE32, ACT_NONE, rows_gemm(r.pooled, D, r.w.proj_t, r.w.proj_b, r.emb, E, B, E, D),
                    st),
        "proj gemm");
  check(launch_l2norm(r.emb, d_out, B, E, st), "l2norm");
}

// SigLIP tail (timm VisionTransformer.norm + AttentionPoolLatent, timm_proj "none"):
// LN(all tokens) -> [k|v] GEMM -> MAP attention with the precomputed latent query -> proj
// -> y + MLP(LN(y)) -> L2 normalise.  Scratch: h (tokens, then the pooled LN), big ([k|v],
// then the MLP hidden), pooled (attention output), x's first B rows (y, f32).
void head_map(const clipgpu_engine& e, const Replica& r, int B, float* d_out, hipStream_t st) {
  const TowerSpec& s = e.spec;
  const int D = s.width, T = s.tokens(), M = mlp_pad(s);
  const MapHeadW& mw = r.w.map;
  ProfScope ps(e, PC_HEAD, st);
  check(launch_ln_rows(e.dt, r.x, 0, r.w.lnpost_w, r.w.lnpost_b, s.ln_eps, r.h, B * T, D, st), "norm");
  check(launch_gemm(e.dt, A_ROWS, EPI_STORE16, ACT_NONE, rows_gemm(r.h, D, mw.wkv, mw.bkv, r.big, 2 * D, B * T, 2 * D, D),
                    st), "attn_pool kv gemm");
  check(launch_map_attention(e.dt, mw.q, r.big, r.pooled, B, T, s.heads, D, st), "attn_pool attention");
  check(launch_gemm(e.dt, A_ROWS, EPI_STORE32, ACT_NONE, rows_gemm(r.pooled, D, mw.wproj, mw.bproj, r.x, D, B, D, D), st),
        "attn_pool proj gemm");
  check(launch_ln_rows(e.dt, r.x, 0, mw.norm_w, mw.norm_b, s.ln_eps, r.h, B, D, st), "attn_pool norm");
  check(launch_gemm(e.dt, A_ROWS, EPI_STORE16, s.act, rows_gemm(r.h, D, mw.w1, mw.b1, r.big, M, B, M, D), st),
        "attn_pool fc1 gemm");
  check(launch_gemm(e.dt, A_ROWS, EPI_RESID, ACT_NONE, rows_gemm(r.big, M, mw.w2, mw.b2, r.x, D, B, D, M), st),
        "attn_pool fc2 gemm");
  check(launch_l2norm((const float*)r.x, d_out, B, D, st), "l2norm");
}

// asrc: A_IMG_F32 (pixels = normalised f32 NCHW) or A_IMG_U8 (NHWC u8 + mean/std)
void vision_forward(const clipgpu_engine& e, const Replica& r, const void* pixels, int asrc, const float* mean,
                    const float* stdv, int B, float* d_out, hipStream_t st) {
  const TowerSpec& s = e.spec;
  const int D = s.width, G = s.grid(), P = s.patch_size, Kp = kpatch_pad(s);
  { ProfScope ps(e, PC_PATCH, st);
    // conv1 = patch rows (16-bit, staged in `big`) x conv_w^T, epilogue + bias + pos -> x
    check(launch_patch_rows(e.dt, asrc, pixels, mean, stdv, r.big, B, s.image_size, P, kpatch(s), Kp, st),
          "patch rows");
    GemmParams g = rows_gemm(r.big, Kp, r.w.conv_w, r.w.conv_b, r.x, D, B * G * G, D, Kp);
    g.G = G;
    g.pos = r.w.pos;
    g.cls = s.cls() ? 1 : 0;
    g.x16 = e.x16 ? 1 : 0;
    g.tile = 2 * B * s.tokens() > e.tuned_rows ? e.tile_patch : TILE_AUTO;
    check(launch_gemm(e.dt, A_ROWS, EPI_PATCH, ACT_NONE, g, st), "patch gemm"); }
  if (s.family == FAMILY_SIGLIP) {  // no class token, no pre-norm: x = patches + bias + pos
    { ProfScope ps(e, PC_STEM, st);
      check(launch_ln_rows(e.dt, r.x, e.x16, r.w.layers[0].ln1_w, r.w.layers[0].ln1_b, s.ln_eps, r.h, B * s.tokens(), D, st,
                           ln_q(e, 0, GS_QKV, r.hs)),
            "ln_1"); }
    trunk(e, r, B, 0, nullptr, st, s.tokens());
    head_map(e, r, B, d_out, st);
    return;
  }
  {
  ProfScope ps(e, PC_STEM, st);
  check(launch_vision_embed_ln(e.dt, r.x, e.x16, r.w.cls, r.w.pos, r.w.lnpre_w, r.w.lnpre_b, r.w.layers[0].ln1_w,
                               r.w.layers[0].ln1_b, s.ln_eps, e.lnf ? nullptr : r.h, B, s.tokens(), D, st,
                               ln_q(e, 0, GS_QKV, r.hs), r.xs),
        "embed+ln_pre");
  }
  head(e, r, B, trunk(e, r, B, 0, nullptr, st, s.tokens()), d_out, st);
}

// T: tokens per sequence in d_ids ([B][T]): the context length, or a trimmed length (every
// sequence's EOT inside the first T tokens, clipgpu_embed_tokens) -- causal attention makes
// the tokens after a sequence's EOT invisible to its pooled row.
void text_forward(const clipgpu_engine& e, const Replica& r, const int64_t* d_ids, int B, float* d_out,
                  hipStream_t st, int T = 0) {
  const TowerSpec& s = e.spec;
  if (T <= 0) T = s.context_length;
  {
  ProfScope ps(e, PC_STEM, st);
  check(launch_text_embed_ln(e.dt, d_ids, r.w.tok, r.w.pos, r.w.layers[0].ln1_w, r.w.layers[0].ln1_b, s.ln_eps,
                             r.x, e.x16, e.lnf ? nullptr : r.h, B, T, s.width, s.vocab_size, st,
                             ln_q(e, 0, GS_QKV, r.hs), r.xs),
        "token embed+ln_1");
  }
  // CLIP: causal, the EOT (argmax id) row pooled; SigLIP2: no mask, the last position pooled
  head(e, r, B, trunk(e, r, B, s.causal ? 1 : 0, s.pool_last ? nullptr : d_ids, st, T, s.pool_last ? T - 1 : 0),
       d_out, st);
}

// The replica's workspace seen from batch row b0: every activation buffer is
// batch-major, so a sub-batch is a pointer offset.
Replica lane_view(const clipgpu_engine& e, const Replica& r, int b0) {
  const TowerSpec& s = e.spec;
  const size_t rows = (size_t)b0 * s.tokens(), D = s.width;
  const size_t wide = big_wide(s);
  Replica v = r;
  v.x = (char*)r.x + rows * D * xbytes(e);
  v.xs = r.xs + rows * 2;
  v.h = (char*)r.h + rows * D * 2;
  v.big = (char*)r.big + rows * wide * 2;
  if (r.hs) v.hs = r.hs + rows * D / 32;
  if (r.bigs) v.bigs = r.bigs + rows * (size_t)mlp_pad(s) / 32;
  v.pooled = (char*)r.pooled + (size_t)b0 * D * 2;
  v.emb = r.emb + (size_t)b0 * s.embed_dim;
  return v;
}

// Batch split for `lanes` concurrent sub-batches: lane i gets rows [b0, b1).
inline void lane_range(int B, int lanes, int i, int& b0, int& b1) {
  b0 = (int)((long)B * i / lanes);
  b1 = (int)((long)B * (i + 1) / lanes);
}

inline int lanes_for(const clipgpu_engine& e, int B) {
  return B < 8 * e.dev_lanes ? 1 : e.dev_lanes;  // small batches gain nothing from lanes
}

// Runs fwd(view, b0, n, stream) on each lane, forked from and joined back to `st`.
// While profiling, the same per-lane launches run one after another on `st`, so
// each kernel's HIP-event time is its own (same shapes as the concurrent run).
template <typename F>
void run_lanes(const clipgpu_engine& e, const Replica& r, int B, hipStream_t st, F fwd) {
  const int L = lanes_for(e, B);
  // profiling serializes the lanes (each event pair times one kernel alone), unless the mask asks
  // for the concurrent regime (CLIPGPU_PROFILE_CONCURRENT)
  const bool serial = e.prof.mask != 0 && !(e.prof.mask & CLIPGPU_PROFILE_CONCURRENT);
  if (L == 1 || serial) {
    for (int i = 0; i < L; ++i) {
      int b0, b1;
      lane_range(B, L, i, b0, b1);
      fwd(lane_view(e, r, b0), b0, b1 - b0, st);
    }
    return;
  }
  HIP_CHECK(hipEventRecord(r.fork, st));
  for (int i = 0; i < L; ++i) {
    int b0, b1;
    lane_range(B, L, i, b0, b1);
    HIP_CHECK(hipStreamWaitEvent(r.lane[i], r.fork, 0));
    fwd(lane_view(e, r, b0), b0, b1 - b0, r.lane[i]);
    HIP_CHECK(hipEventRecord(r.join[i], r.lane[i]));
  }
  for (int i = 0; i < L; ++i) HIP_CHECK(hipStreamWaitEvent(st, r.join[i], 0));
}

// Runs body(stream) as a replayed hipGraph (captured on first use of `key`).  The capture
// and replay stream is `st` when it is one of the replica's own streams, else the replica's
// stream, forked from and joined back to `st` by events (a caller's stream may be the
// legacy null stream, which cannot be captured).  Profiling (per-launch events) and
// clipgpu_options.graphs = -1 run the body directly.
template <typename F>
void run_graph(const clipgpu_engine& e, const Replica& r, const std::vector<uint64_t>& key_in, hipStream_t st, F body) {
  if (!e.graphs || e.prof.mask || !r.graphs) {
    body(st);
    return;
  }
  bool own = st == r.stream;
  for (int i = 0; i < 4; ++i) own = own || (st != nullptr && st == r.lane[i]);
  hipStream_t gs = own ? st : r.stream;
  GraphCache& gc = *r.graphs;
  hipGraphExec_t exec = nullptr;
#ifdef CLIPGPU_ABLATE
  std::vector<uint64_t> key = key_in;
  key.push_back(0xAB1A7E00u | g_ablate);
#else
  const std::vector<uint64_t>& key = key_in;
#endif
  ++gc.clock;
  for (auto& en : gc.entries)
    if (en.key == key) {
      exec = en.exec;
      en.last_use = gc.clock;
    }
  if (!exec && gc.entries.size() >= GraphCache::kMax) {  // evict the least recently used graph
    HIP_CHECK(hipStreamSynchronize(r.stream));
    for (int i = 0; i < 4; ++i)
      if (r.lane[i]) HIP_CHECK(hipStreamSynchronize(r.lane[i]));
    if (!own) HIP_CHECK(hipStreamSynchronize(st));
    size_t lru = 0;
    for (size_t i = 1; i < gc.entries.size(); ++i)
      if (gc.entries[i].last_use < gc.entries[lru].last_use) lru = i;
    (void)hipGraphExecDestroy(gc.entries[lru].exec);
    gc.entries.erase(gc.entries.begin() + (long)lru);
  }
  if (!own) {
    HIP_CHECK(hipEventRecord(r.gin, st));
    HIP_CHECK(hipStreamWaitEvent(gs, r.gin, 0));
  }
  if (!exec) {
    hipGraph_t g = nullptr;
    HIP_CHECK(hipStreamBeginCapture(gs, hipStreamCaptureModeRelaxed));
    try {
      body(gs);
    } catch (...) {
      (void)hipStreamEndCapture(gs, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    HIP_CHECK(hipStreamEndCapture(gs, &g));
    const hipError_t ie = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIP_CHECK(ie);
    gc.entries.push_back({key, exec, gc.clock});
  }
  HIP_CHECK(hipGraphLaunch(exec, gs));
  if (!own) {
    HIP_CHECK(hipEventRecord(r.gout, gs));
    HIP_CHECK(hipStreamWaitEvent(st, r.gout, 0));
  }
}

inline uint64_t fbits(const float* v, int i) {
  uint32_t u = 0;
  if (v) std::memcpy(&u, v + i, 4);
  return u;
}

void vision_forward_lanes(const clipgpu_engine& e, const Replica& r, const void* pixels, int asrc, const float* mean,
                          const float* stdv, int B, float* d_out, hipStream_t st) {
  const size_t S = e.spec.image_size;
  const size_t row_bytes = 3 * S * S * (asrc == A_IMG_F32 ? 4 : 1);
  const int E = e.spec.embed_dim;
  run_lanes(e, r, B, st, [&](const Replica& v, int b0, int n, hipStream_t ls) {
    vision_forward(e, v, (const char*)pixels + b0 * row_bytes, asrc, mean, stdv, n, d_out + (size_t)b0 * E, ls);
  });
}

void text_forward_lanes(const clipgpu_engine& e, const Replica& r, const int64_t* d_ids, int B, float* d_out,
                        hipStream_t st) {
  const int E = e.spec.embed_dim, T = e.spec.context_length;
  run_lanes(e, r, B, st, [&](const Replica& v, int b0, int n, hipStream_t ls) {
    text_forward(e, v, d_ids + (size_t)b0 * T, n, d_out + (size_t)b0 * E, ls);
  });
}

// Second tuning pass over whole forwards: the per-site autotune times each GEMM alone, but
// in the forward two lanes' kernels share the chip, so a tile that wins alone can lose there.
// Coordinate descent: for each trunk site, try every other tile with the rest fixed and keep
// it if the concurrent-lane forward at max_batch gets >= 1 % faster.  Inputs are the zeroed
// staging buffer (timing only).  clipgpu_options.tuning = 2 skips it; pinned tiles skip it.
void tune_forward(clipgpu_engine& e, Replica& r) {
  if (e.tuning != 1 || tiles_pinned(e) || e.max_batch < 64 || e.mx) return;
  const int B = e.max_batch;
  hipEvent_t a, b;
  HIP_CHECK(hipEventCreate(&a));
  HIP_CHECK(hipEventCreate(&b));
  auto fwd = [&]() {
    if (e.spec.tower == TOWER_VISION)
      vision_forward_lanes(e, r, r.in, A_IMG_F32, nullptr, nullptr, B, r.out, r.stream);
    else
      text_forward_lanes(e, r, (const int64_t*)r.in, B, r.out, r.stream);
  };
  auto time_once = [&]() {
    fwd();
    HIP_CHECK(hipEventRecord(a, r.stream));
    for (int i = 0; i < 3; ++i) fwd();
    HIP_CHECK(hipEventRecord(b, r.stream));
    HIP_CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
  };
  // the better of two timings: one disturbed measurement does not decide a choice
  auto time_fwd = [&]() { return std::min(time_once(), time_once()); };
  float best = time_fwd();
  if (!e.lanes_pinned && e.lanes > 1) {  // lanes: the configured count, or the whole batch on one stream
    int keep_tiles[GS_N], keep_patch = e.tile_patch, keep_rows = e.tuned_rows;
    for (int i = 0; i < GS_N; ++i) keep_tiles[i] = e.tile[i];
    e.dev_lanes = 1;
    autotune_tiles(e, r);
    const float one = time_fwd();
    if (one < 0.99f * best) {
      best = one;
    } else {  // back to the lanes and their tiles
      e.dev_lanes = e.lanes;
      for (int i = 0; i < GS_N; ++i) e.tile[i] = keep_tiles[i];
      e.tile_patch = keep_patch;
      e.tuned_rows = keep_rows;
    }
  }
  for (int site = 0; site < GS_N; ++site) {
    const int keep = e.tile[site];
    for (int t : kTuneCands) {
      if (t == keep) continue;
      const int prev = e.tile[site];
      e.tile[site] = t;
      const float ms = time_fwd();
      if (ms < 0.99f * best) {  // confirm against the kept tile re-timed before and after the
        e.tile[site] = prev;    // candidate's second timing: neither a lucky timing nor a clock
        const float kept = time_fwd();  // drift between timings decides the choice
        e.tile[site] = t;
        const float again = time_fwd();
        e.tile[site] = prev;
        const float kept2 = time_fwd();
        if (again < 0.99f * std::min(kept, kept2)) {
          e.tile[site] = t;
          best = std::min(ms, again);
        } else {
          best = std::min(best, std::min(kept, kept2));
        }
      } else {
        e.tile[site] = prev;
      }
    }
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
}

enum InKind { IN_F32 = 0, IN_U8 = 1, IN_IDS = 2 };

// Row source of a host entry point: a contiguous array (row i at in + i * row_bytes), or one pointer per
// row (`rows`: the decoded-image entry point's S x S images, which already are the u8 NHWC rows).
struct HostRows {
  const char* in = nullptr;
  const void* const* rows = nullptr;
  size_t row_bytes = 0;
};

// Caller-registered host ranges (clipgpu_host_register): process-wide, hipHostRegister'ed.
constexpr size_t kHostPage = 4096;
struct HostRanges {
  std::mutex mu;
  std::vector<std::pair<uintptr_t, size_t>> r;  // (base, bytes)
};
HostRanges& host_ranges() {
  static HostRanges h;
  return h;
}
// Is [p, p + n) inside one registered range?
bool host_registered(const void* p, size_t n) {
  HostRanges& h = host_ranges();
  std::lock_guard<std::mutex> lk(h.mu);
  const uintptr_t a = (uintptr_t)p;
  for (const auto& rg : h.r)
    if (a >= rg.first && a + n <= rg.first + rg.second) return true;
  return false;
}

// The fixed partition of a round's max_batch rows into host-path chunks: part[0] = 0 < part[1] <
// ... < part[C] = MB, `lanes` even chunks.  Measured on the bench's ViT-B/32 u8 batch of 256
// (tools/host_plan_ab.py, profiles/r04_host_plan_ab.jsonl): two halves beat a small first chunk
// (64 or 96 rows) and three- or four-chunk plans, whose small forwards run far below the full
// batch's rate.
std::vector<int> host_chunks(const clipgpu_engine& e, InKind kind) {
  const int MB = e.max_batch, L = e.lanes;
  if (!e.host_part.empty() && kind != IN_IDS) return e.host_part;
  std::vector<int> part{0};
  for (int i = 1; i < L; ++i) part.push_back((int)(((long)MB * i + L - 1) / L));
  part.push_back(MB);
  return part;
}

// The second host-path buffer set of a replica (multi-round host calls), allocated once.
void ensure_host_set2(const clipgpu_engine& e, Replica& r) {
  if (r.in2) return;
  const size_t B = (size_t)((e.max_batch + e.lanes - 1) / e.lanes * e.lanes);
  HIP_CHECK(hipMalloc(&r.in2, B * e.in_bytes_per_row));
  HIP_CHECK(hipHostMalloc(&r.pin_in2, B * e.in_bytes_per_row, hipHostMallocDefault));
  HIP_CHECK(hipHostMalloc((void**)&r.pin_out2, B * (size_t)e.spec.embed_dim * 4, hipHostMallocDefault));
  HIP_CHECK(hipMalloc((void**)&r.out2, B * (size_t)e.spec.embed_dim * 4));
  for (int i = 0; i < 4; ++i) {
    HIP_CHECK(hipEventCreateWithFlags(&r.done2[i], hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&r.copied2[i], hipEventDisableTiming));
  }
}

// Host-buffer forward over a row range of one replica.  Each round of up to max_batch rows is cut
// by host_chunks' partition; chunk k of a round uses rows [part[k], part[k + 1]) of the
// max_batch-row device buffers, workspace (lane_view) and pinned staging, so chunks of one round
// never share memory and chunk k of the next round reuses only chunk k's rows, after chunk k's D2H
// event.  The H2Ds go in chunk order on the replica's copy stream (the first chunk gets the whole
// link); chunk k's forward runs on lane stream k % lanes once its copy event has fired, so the
// transfer of chunk k + 1 overlaps the forward of chunk k, and forwards of different lanes
// overlap each other.  Inputs are DMA'd straight from a caller-registered range
// (clipgpu_host_register) or staged through pinned memory by the copy pool in pieces of whole rows
// (kStagePiece), each piece's H2D issued as soon as it is packed, so a chunk's transfer runs under the
// packing of its later pieces; outputs are written straight into a registered range, or staged.
// A range of more than max_batch rows alternates its rounds between two buffer sets (device input
// rows, pinned staging, events): round i's host copy and H2D are issued while round i - 1's forward
// runs, and a set is reused two rounds later, after its round's D2H event -- so every round but the
// first starts its forward with its input already on the device.  Each set also
// has its own device embedding rows, copied back on the second copy stream once the forward has ended,
// so a lane's next forward starts right behind its last one.  Each round runs the same forward on the
// same rows as a call of its own: the outputs are bit-identical.
// (Round 6 removed the schedules measured and not kept -- lockstep, joined and device-path rounds, D2H
// on the copy or lane streams, split and pulled H2Ds; DESIGN.md §10 keeps their numbers.)
constexpr size_t kStagePiece = 4u << 20;

void run_host_shard(clipgpu_engine& e, Replica& r, InKind kind, const HostRows& src, int64_t b0, int64_t b1,
                    const float* mean, const float* stdv, float* out, int tokens = 0) {
  HIP_CHECK(hipSetDevice(r.device));
  const int E = e.spec.embed_dim, L = e.lanes, MB = e.max_batch;
  const size_t rb = src.row_bytes;
  const bool direct_in = src.rows == nullptr && host_registered(src.in + b0 * rb, (size_t)(b1 - b0) * rb);
  const bool direct_out = host_registered(out + b0 * E, (size_t)(b1 - b0) * E * 4);
  const std::vector<int> part = host_chunks(e, kind);
  const int C = (int)part.size() - 1;
  const bool two_sets = b1 - b0 > MB;
  if (two_sets) ensure_host_set2(e, r);
  struct Pending { int64_t c0 = -1; int n = 0; };
  Pending pend[2][4];
  float* const pin_out_set[2] = {r.pin_out, r.pin_out2};
  hipEvent_t* const done_set[2] = {r.done, r.done2};
  auto drain = [&](int set, int k) {
    if (pend[set][k].c0 < 0) return;
    HIP_CHECK(hipEventSynchronize(done_set[set][k]));
    if (!direct_out)
      std::memcpy(out + pend[set][k].c0 * E, pin_out_set[set] + (size_t)part[k] * E, (size_t)pend[set][k].n * E * 4);
    pend[set][k].c0 = -1;
  };
  const int rows_per_piece = (int)std::max<size_t>(1, kStagePiece / rb);
  int round = 0;
  for (int64_t c0 = b0; c0 < b1; ++round) {
    const int set = two_sets ? (round & 1) : 0;
    char* const in_base = (char*)(set ? r.in2 : r.in);
    char* const pin_in_base = (char*)(set ? r.pin_in2 : r.pin_in);
    hipEvent_t* const done = set ? r.done2 : r.done;
    hipEvent_t* const copied = set ? r.copied2 : r.copied;
    const int R = (int)std::min<int64_t>(MB, b1 - c0);  // rows of this round
    int off = 0;
    for (int k = 0; k < C && off < R; ++k) {
      const int cap = part[k + 1] - part[k];
      // a round of at least half of max_batch spreads over the chunks in proportion to the
      // partition; a shorter one fills them in order (a small batch is one forward)
      int n = 2 * R < MB ? R - off
              : k + 1 == C ? R - off : (int)(((long)R * part[k + 1] + MB - 1) / MB - off);
      n = std::max(0, std::min(n, cap));
      if (n == 0) continue;
      const int64_t rc = c0 + off;
      drain(set, k);  // this set's round before last: its D2H (so also its H2D and forward) done
      hipStream_t st = r.lane[k % L] ? r.lane[k % L] : r.stream;
      char* din = in_base + (size_t)part[k] * rb;
      float* dout = (set ? r.out2 : r.out) + (size_t)part[k] * E;
      if (direct_in) {
        HIP_CHECK(hipMemcpyAsync(din, src.in + rc * rb, (size_t)n * rb, hipMemcpyHostToDevice, r.copy));
      } else {
        char* pin = pin_in_base + (size_t)part[k] * rb;
        for (int p0 = 0; p0 < n; p0 += rows_per_piece) {
          const int pn = std::min(rows_per_piece, n - p0);
          char* pp = pin + (size_t)p0 * rb;
          if (src.rows) pool_gather(pp, src.rows + rc + p0, rb, pn);
          else pool_memcpy(pp, src.in + (rc + p0) * rb, (size_t)pn * rb);
          HIP_CHECK(hipMemcpyAsync(din + (size_t)p0 * rb, pp, (size_t)pn * rb, hipMemcpyHostToDevice, r.copy));
        }
      }
      HIP_CHECK(hipEventRecord(copied[k], r.copy));
      HIP_CHECK(hipStreamWaitEvent(st, copied[k], 0));
      const Replica v = lane_view(e, r, part[k]);
      run_graph(e, r,
                {(uint64_t)(10 + kind), (uint64_t)k, (uint64_t)n, fbits(mean, 0), fbits(mean, 1), fbits(mean, 2),
                 fbits(stdv, 0), fbits(stdv, 1), fbits(stdv, 2), (uint64_t)tokens, (uint64_t)part[k], (uint64_t)set,
                 (uint64_t)(uintptr_t)dout},
                st, [&](hipStream_t gs) {
                  if (kind == IN_IDS)
                    text_forward(e, v, (const int64_t*)din, n, dout, gs, tokens);
                  else
                    vision_forward(e, v, din, kind == IN_F32 ? A_IMG_F32 : A_IMG_U8, mean, stdv, n, dout, gs);
                });
      float* dst = direct_out ? out + rc * E : pin_out_set[set] + (size_t)part[k] * E;
      if (two_sets) {  // the forward's end, then the D2H on the second copy stream
        HIP_CHECK(hipEventRecord(done[k], st));
        HIP_CHECK(hipStreamWaitEvent(r.copy2, done[k], 0));
        HIP_CHECK(hipMemcpyAsync(dst, dout, (size_t)n * E * 4, hipMemcpyDeviceToHost, r.copy2));
        HIP_CHECK(hipEventRecord(done[k], r.copy2));
      } else {
        HIP_CHECK(hipMemcpyAsync(dst, dout, (size_t)n * E * 4, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipEventRecord(done[k], st));
      }
      pend[set][k].c0 = rc;
      pend[set][k].n = n;
      off += n;
    }
    c0 += R;
  }
  for (int set = 0; set < 2; ++set)
    for (int k = 0; k < C; ++k) drain(set, k);
}

void run_host(clipgpu_engine& e, InKind kind, const HostRows& src, int64_t B, const float* mean, const float* stdv,
              float* out, int tokens = 0) {
  const int G = (int)e.reps.size();
  if (G == 1) {
    run_host_shard(e, e.reps[0], kind, src, 0, B, mean, stdv, out, tokens);
    return;
  }
  // Contiguous row blocks, rank order == input order.
  std::vector<std::thread> th;
  std::vector<std::string> errs(G);
  std::vector<int> codes(G, 0);
  for (int g = 0; g < G; ++g) {
    const int64_t b0 = B * g / G, b1 = B * (g + 1) / G;
    if (b0 == b1) continue;
    th.emplace_back([&, g, b0, b1]() {
      try {
        run_host_shard(e, e.reps[g], kind, src, b0, b1, mean, stdv, out, tokens);
      } catch (const ClipErr& ex) {
        codes[g] = ex.code;
        errs[g] = ex.what();
      } catch (const std::exception& ex) {
        codes[g] = CLIPGPU_ERR_DEVICE;
        errs[g] = ex.what();
      }
    });
  }
  for (auto& t : th) t.join();
  for (int g = 0; g < G; ++g)
    if (codes[g]) throw ClipErr(codes[g], "device " + std::to_string(e.reps[g].device) + ": " + errs[g]);
}

// ---- decoded RGB8 images -> embeddings, crop/resize on the GPU -------------------------
// Host: per image a ResizePlan (the same fixed-point tables as the host resize); device:
// launch_resize into the slot's u8 NHWC input rows, then the u8 vision forward (normalise
// + patch rows + trunk).  Chunks of <= one lane's rows (and <= kChunkRawBytes of source
// pixels) pipelined over the lane slots as run_host_shard does.
constexpr size_t kChunkRawBytes = 256u << 20;

// The staged source of an image is only the window its resize reads (round 6): the horizontal pass reads
// source rows [yfirst, yfirst + th) and, over all its outputs, columns [x0, x1) -- a 640x480 image cropped
// to its centre square needs 486 of its 640 columns; a vertical-only plan (width already S) reads rows
// [y0, y1).  The descriptor and the tap bounds are shifted to the window, so every output reads the same
// pixels with the same coefficients (bit-identical to the host resize).
struct ResizeBatch {
  std::vector<ResizeImage> d;
  std::vector<int> ints;
  std::vector<size_t> raw_off;  // per image, in the raw region
  struct Window { int y0, rows, x0, cols; };
  std::vector<Window> win;      // per image: the source window staged
  size_t raw_bytes = 0, tmp_bytes = 0;
  int max_th = 0;
};

inline size_t align16(size_t n) { return (n + 15) & ~size_t(15); }

ResizeBatch plan_resize_batch(int S, const std::string& interp, const std::string& mode, const int* W, const int* H,
                              int64_t i0, int n) {
  ResizeBatch b;
  b.d.resize(n);
  b.raw_off.resize(n);
  b.win.resize(n);
  for (int i = 0; i < n; ++i) {
    const ResizePlan p = make_resize_plan(W[i0 + i], H[i0 + i], S, interp, mode);
    ResizeImage& d = b.d[i];
    d.W = p.W;
    d.th = p.need_h ? p.th : 0;
    d.yfirst = p.yfirst;
    d.need_h = p.need_h;
    d.need_v = p.need_v;
    d.h_ksize = p.h.ksize;
    d.v_ksize = p.v.ksize;
    d.h_prec = p.h.prec;
    d.v_prec = p.v.prec;
    auto put = [&](const std::vector<int>& v) {
      const long off = (long)b.ints.size();
      b.ints.insert(b.ints.end(), v.begin(), v.end());
      return off;
    };
    ResizeBatch::Window w{0, p.H, 0, p.W};
    std::vector<int> hb = p.h.bounds, vb = p.v.bounds;
    if (p.need_h && p.th > 0 && !hb.empty()) {  // rows [yfirst, yfirst + th), the columns the taps read
      int x0 = hb[0], x1 = hb[0] + hb[1];
      for (size_t o = 0; o + 1 < hb.size(); o += 2) {
        x0 = std::min(x0, hb[o]);
        x1 = std::max(x1, hb[o] + hb[o + 1]);
      }
      for (size_t o = 0; o < hb.size(); o += 2) hb[o] -= x0;
      w = {p.yfirst, p.th, x0, x1 - x0};
      d.W = w.cols;
      d.yfirst = 0;
    } else if (!p.need_h && p.need_v && !vb.empty()) {  // the rows the vertical taps read, all S columns
      int y0 = vb[0], y1 = vb[0] + vb[1];
      for (size_t o = 0; o + 1 < vb.size(); o += 2) {
        y0 = std::min(y0, vb[o]);
        y1 = std::max(y1, vb[o] + vb[o + 1]);
      }
      for (size_t o = 0; o < vb.size(); o += 2) vb[o] -= y0;
      w = {y0, y1 - y0, 0, p.W};
    }
    b.win[i] = w;
    d.h_bounds = put(hb);
    d.h_coef = put(std::vector<int>(p.h.k.begin(), p.h.k.end()));
    d.v_bounds = put(vb);
    d.v_coef = put(std::vector<int>(p.v.k.begin(), p.v.k.end()));
    b.raw_off[i] = b.raw_bytes;
    d.src = (long)b.raw_bytes;  // relative to the raw region
    b.raw_bytes = align16(b.raw_bytes + (size_t)w.rows * w.cols * 3);
    d.tmp = (long)b.tmp_bytes;
    if (p.need_h) b.tmp_bytes = align16(b.tmp_bytes + (size_t)p.th * S * 3);
    b.max_th = std::max(b.max_th, d.th);
  }
  return b;
}

// Copy tasks that stage image i's window (src: its full [H][W][3] pixels, W its width) at dst.
void add_window_tasks(std::vector<CopyTask>& t, const ResizeBatch& b, int i, char* dst, const uint8_t* src, int W) {
  const ResizeBatch::Window& w = b.win[i];
  add_copy_tasks_2d(t, dst, src + ((size_t)w.y0 * W + w.x0) * 3, (size_t)w.cols * 3, (size_t)w.rows, (size_t)W * 3);
}

void grow_pinned(char*& p, size_t& cap, size_t need) {
  if (need <= cap) return;
  if (p) HIP_CHECK(hipHostFree(p));
  p = nullptr;
  cap = 0;
  HIP_CHECK(hipHostMalloc((void**)&p, need, hipHostMallocDefault));
  cap = need;
}
template <typename P>
void grow_device(P*& p, size_t& cap, size_t need) {
  if (need <= cap) return;
  if (p) HIP_CHECK(hipFree(p));
  p = nullptr;
  cap = 0;
  HIP_CHECK(hipMalloc((void**)&p, need));
  cap = need;
}

// Chunks alternate over the lane slots; per chunk: the resize plans' tables and the source images are
// packed into the slot's pinned staging by the copy pool, in pieces of whole images (kStagePiece) whose
// H2Ds go on the copy stream as soon as each is packed (round 6; round 5 spawned std::threads per chunk
// and ran the H2D on the lane stream), then on the lane: the resize kernels into the slot's u8 rows and
// the u8 forward.  The packing of chunk j + 1 runs while chunk j transfers and computes.
void run_images_shard(clipgpu_engine& e, Replica& r, const uint8_t* const* images, const int* W, const int* H,
                      int64_t b0, int64_t b1, float* out) {
  HIP_CHECK(hipSetDevice(r.device));
  const int E = e.spec.embed_dim, L = e.lanes, S = e.spec.image_size;
  const int rows = (e.max_batch + L - 1) / L;  // rows per slot
  struct Pending { int64_t c0 = -1; int n = 0; };
  Pending pend[4];
  auto drain = [&](int k) {
    if (pend[k].c0 < 0) return;
    HIP_CHECK(hipEventSynchronize(r.done[k]));
    std::memcpy(out + pend[k].c0 * E, r.pin_out + (size_t)k * rows * E, (size_t)pend[k].n * E * 4);
    pend[k].c0 = -1;
  };
  int j = 0;
  for (int64_t c0 = b0; c0 < b1; ++j) {
    // chunk: up to `rows` images and kChunkRawBytes of source pixels (at least one image)
    int n = 0;
    size_t raw = 0;
    while (c0 + n < b1 && n < rows) {
      const size_t sz = (size_t)W[c0 + n] * H[c0 + n] * 3;
      if (n > 0 && raw + sz > kChunkRawBytes) break;
      raw += sz;
      ++n;
    }
    const int k = j % L;
    drain(k);  // slot k's previous chunk (its H2D, resize, forward and D2H) is done
    hipStream_t st = r.lane[k] ? r.lane[k] : r.stream;
    const ResizeBatch b = plan_resize_batch(S, e.pre.interpolation, e.pre.resize_mode, W, H, c0, n);
    const size_t desc_bytes = align16(b.d.size() * sizeof(ResizeImage));
    const size_t ints_bytes = align16(b.ints.size() * sizeof(int));
    const size_t head = desc_bytes + ints_bytes, total = head + b.raw_bytes;
    Replica::ImageSlot& sl = r.islot[k];
    grow_pinned(sl.pin, sl.pin_cap, total);
    grow_device(sl.dev, sl.dev_cap, total);
    grow_device(sl.tmp, sl.tmp_cap, std::max<size_t>(b.tmp_bytes, 16));
    std::memcpy(sl.pin, b.d.data(), b.d.size() * sizeof(ResizeImage));
    std::memcpy(sl.pin + desc_bytes, b.ints.data(), b.ints.size() * sizeof(int));
    HIP_CHECK(hipMemcpyAsync(sl.dev, sl.pin, head, hipMemcpyHostToDevice, r.copy));
    char* const raw_pin = sl.pin + head;
    for (int i0 = 0; i0 < n;) {  // pieces of whole images
      int i1 = i0 + 1;
      while (i1 < n && b.raw_off[i1] - b.raw_off[i0] < kStagePiece) ++i1;
      const size_t p0 = b.raw_off[i0], p1 = i1 < n ? b.raw_off[i1] : b.raw_bytes;
      std::vector<CopyTask> tasks;
      for (int i = i0; i < i1; ++i) add_window_tasks(tasks, b, i, raw_pin + b.raw_off[i], images[c0 + i], W[c0 + i]);
      pool_copy(tasks);
      HIP_CHECK(hipMemcpyAsync(sl.dev + head + p0, raw_pin + p0, p1 - p0, hipMemcpyHostToDevice, r.copy));
      i0 = i1;
    }
    HIP_CHECK(hipEventRecord(r.copied[k], r.copy));
    HIP_CHECK(hipStreamWaitEvent(st, r.copied[k], 0));
    uint8_t* din = (uint8_t*)r.in + (size_t)k * rows * e.in_bytes_per_row;  // u8 [n][S][S][3]
    check(launch_resize((const uint8_t*)sl.dev + head, sl.tmp, (const int*)(sl.dev + desc_bytes),
                        (const ResizeImage*)sl.dev, n, b.max_th, S, din, st), "resize");
    float* dout = r.out + (size_t)k * rows * E;
    const Replica v = lane_view(e, r, k * rows);
    run_graph(e, r, {20, (uint64_t)k, (uint64_t)n}, st,
              [&](hipStream_t gs) { vision_forward(e, v, din, A_IMG_U8, e.pre.mean, e.pre.stdv, n, dout, gs); });
    HIP_CHECK(hipMemcpyAsync(r.pin_out + (size_t)k * rows * E, dout, (size_t)n * E * 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipEventRecord(r.done[k], st));
    pend[k].c0 = c0;
    pend[k].n = n;
    c0 += n;
  }
  for (int k = 0; k < L; ++k) drain(k);
}

// Contiguous row blocks over the replicas (rank order == input order), one host thread each.
template <typename F>
void run_sharded(clipgpu_engine& e, int64_t B, F shard) {
  const int G = (int)e.reps.size();
  if (G == 1) {
    shard(e.reps[0], (int64_t)0, B);
    return;
  }
  std::vector<std::thread> th;
  std::vector<std::string> errs(G);
  std::vector<int> codes(G, 0);
  for (int g = 0; g < G; ++g) {
    const int64_t b0 = B * g / G, b1 = B * (g + 1) / G;
    if (b0 == b1) continue;
    th.emplace_back([&, g, b0, b1]() {
      try {
        shard(e.reps[g], b0, b1);
      } catch (const ClipErr& ex) {
        codes[g] = ex.code;
        errs[g] = ex.what();
      } catch (const std::exception& ex) {
        codes[g] = CLIPGPU_ERR_DEVICE;
        errs[g] = ex.what();
      }
    });
  }
  for (auto& t : th) t.join();
  for (int g = 0; g < G; ++g)
    if (codes[g]) throw ClipErr(codes[g], "device " + std::to_string(e.reps[g].device) + ": " + errs[g]);
}

// ---- sharded forward + the RCCL all-gather of the embedding rows ----------
// Every rank embeds its own contiguous block of rows[rank] rows into its slot of a [sum rows][E]
// output on its device, then one collective leaves the whole matrix, in rank order, on every
// rank: an in-place ncclAllGather when all blocks are equal, else (ragged blocks) one in-place
// ncclBroadcast per non-empty block inside a group.  `local` is replica i = rank rank0 + i.
// The multi-device handle's communicator, created on its first gathered call (clipgpu_create_ex).
void ensure_comm(clipgpu_engine& e) {
  if (!e.comm_pending) return;
  std::vector<ncclComm_t> comms(e.comm_devs.size());
  NCCL_CHECK(ncclCommInitAll(comms.data(), (int)comms.size(), e.comm_devs.data()));
  for (size_t i = 0; i < comms.size(); ++i) e.reps[i].comm = comms[i];
  e.comm_pending = false;
}

// Host-side plan of a gathered call (no GPU; clipgpu_test_gather_plan checks it on the CPU):
// off[r] = first output row of rank r's block (rank order), equal = every block the same size
// (one ncclAllGather; else one ncclBroadcast per non-empty block), and per local replica the
// forward chunks of at most max_batch rows, each written at its rows of the output.
struct GatherPlan {
  std::vector<int64_t> off;
  bool equal = true;
};
GatherPlan plan_gather(int nr, const int64_t* rows) {
  GatherPlan g;
  g.off.assign((size_t)nr + 1, 0);
  for (int r = 0; r < nr; ++r) {
    if (rows[r] < 0) throw ClipErr(CLIPGPU_ERR_INVALID, "negative row count");
    g.off[r + 1] = g.off[r] + rows[r];
    g.equal = g.equal && rows[r] == rows[0];
  }
  if (g.off[nr] == 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");
  return g;
}

template <typename Fwd>
void sharded_gather(clipgpu_engine& e, const int64_t* rows, float* const* d_out, void* const* streams, Fwd fwd) {
  const int nr = e.comm_nranks, E = e.spec.embed_dim, G = (int)e.reps.size();
  if (nr <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "no communicator: create the handle over distinct devices "
                                                  "or call clipgpu_comm_init_rank first");
  const GatherPlan plan = plan_gather(nr, rows);
  const std::vector<int64_t>& off = plan.off;
  // (test hook clipgpu_test_force_broadcast: the ragged branch with equal blocks)
  const bool equal = plan.equal && !e.force_bcast;
  std::vector<hipStream_t> sts((size_t)G);
  for (int i = 0; i < G; ++i) {
    Replica& r = e.reps[i];
    if (!d_out[i]) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    // NULL array / entry: the legacy default stream of the replica's device, as in the single-device
    // entry points (run_graph forks the forward from it and joins it back; the collective runs on it)
    sts[i] = streams ? (hipStream_t)streams[i] : nullptr;
    const int rank = e.comm_rank0 + i;
    HIP_CHECK(hipSetDevice(r.device));
    for (int64_t c0 = 0; c0 < rows[rank]; c0 += e.max_batch)
      fwd(r, i, c0, (int)std::min<int64_t>(e.max_batch, rows[rank] - c0), d_out[i] + (off[rank] + c0) * E, sts[i]);
  }
  ensure_comm(e);
  NCCL_CHECK(ncclGroupStart());
  for (int i = 0; i < G; ++i) {
    Replica& r = e.reps[i];
    const int rank = e.comm_rank0 + i;
    if (equal) {
      NCCL_CHECK(ncclAllGather(d_out[i] + off[rank] * E, d_out[i], (size_t)rows[rank] * E, ncclFloat, r.comm, sts[i]));
    } else {
      for (int q = 0; q < nr; ++q)
        if (rows[q] > 0)
          NCCL_CHECK(ncclBroadcast(d_out[i] + off[q] * E, d_out[i] + off[q] * E, (size_t)rows[q] * E, ncclFloat, q,
                                   r.comm, sts[i]));
    }
  }
  NCCL_CHECK(ncclGroupEnd());
  // destroy_comms waits for these (the collective runs on the caller's stream, not the handle's)
  for (int i = 0; i < G; ++i) {
    Replica& r = e.reps[i];
    HIP_CHECK(hipSetDevice(r.device));
    if (!r.coll) HIP_CHECK(hipEventCreateWithFlags(&r.coll, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(r.coll, sts[i]));
  }
}

// The handle's communicators: collectives may still be in flight on callers' streams, so each
// replica's last collective (the event recorded behind it on the caller's stream) and the handle's own
// streams are waited for first -- not the whole device, which may run unrelated work (torch, other
// engines); then all of the clique's communicators are finalized inside one group (a one-by-one
// finalize from one thread can block on peers) and destroyed.
void destroy_comms(clipgpu_engine& e) {
  bool any = false;
  for (auto& r : e.reps)
    if (r.comm) {
      (void)hipSetDevice(r.device);
      if (r.coll) (void)hipEventSynchronize(r.coll);
      if (r.stream) (void)hipStreamSynchronize(r.stream);
      for (int i = 0; i < 4; ++i)
        if (r.lane[i]) (void)hipStreamSynchronize(r.lane[i]);
      any = true;
    }
  if (!any) return;
  if (ncclGroupStart() == ncclSuccess) {
    for (auto& r : e.reps)
      if (r.comm) (void)ncclCommFinalize(r.comm);
    (void)ncclGroupEnd();
  }
  for (auto& r : e.reps)
    if (r.comm) {
      (void)ncclCommDestroy(r.comm);
      r.comm = nullptr;
    }
}

void destroy_replica(Replica& r) {
  (void)hipSetDevice(r.device);
  // every stream of the replica (lanes, copy streams: a device-path call's forks may still run) is idle
  // before its memory goes
  (void)hipDeviceSynchronize();
  if (r.arena) (void)hipFree(r.arena);
  if (r.work) (void)hipFree(r.work);
  if (r.pin_in) (void)hipHostFree(r.pin_in);
  if (r.pin_out) (void)hipHostFree(r.pin_out);
  if (r.in2) (void)hipFree(r.in2);
  if (r.pin_in2) (void)hipHostFree(r.pin_in2);
  if (r.pin_out2) (void)hipHostFree(r.pin_out2);
  if (r.out2) (void)hipFree(r.out2);
  if (r.stream) (void)hipStreamDestroy(r.stream);
  if (r.copy) (void)hipStreamDestroy(r.copy);
  if (r.copy2) (void)hipStreamDestroy(r.copy2);
  for (int i = 0; i < 4; ++i) {
    if (r.lane[i]) (void)hipStreamDestroy(r.lane[i]);
    if (r.join[i]) (void)hipEventDestroy(r.join[i]);
    if (r.done[i]) (void)hipEventDestroy(r.done[i]);
    if (r.copied[i]) (void)hipEventDestroy(r.copied[i]);
    if (r.done2[i]) (void)hipEventDestroy(r.done2[i]);
    if (r.copied2[i]) (void)hipEventDestroy(r.copied2[i]);
  }
  if (r.fork) (void)hipEventDestroy(r.fork);
  if (r.gin) (void)hipEventDestroy(r.gin);
  if (r.gout) (void)hipEventDestroy(r.gout);
  if (r.coll) (void)hipEventDestroy(r.coll);
  if (r.graphs) {
    r.graphs->clear();
    delete r.graphs;
  }
  for (auto& sl : r.islot) {
    if (sl.pin) (void)hipHostFree(sl.pin);
    if (sl.dev) (void)hipFree(sl.dev);
    if (sl.tmp) (void)hipFree(sl.tmp);
  }
  r = Replica();
}

}  // namespace
}  // namespace clipgpu

using namespace clipgpu;

extern "C" {

int clipgpu_abi_version(void) { return CLIPGPU_ABI_VERSION; }

int clipgpu_options_init(clipgpu_options* o) {
  return guarded([&]() {
    if (!o) throw ClipErr(CLIPGPU_ERR_INVALID, "opts is NULL");
    std::memset(o, 0, sizeof(*o));
    o->struct_size = sizeof(*o);
  });
}

int clipgpu_create(const char* model_dir, int tower, const int* device_ids, int n_devices, int dtype, int max_batch,
                   clipgpu_engine** out) {
  return clipgpu_create_ex(model_dir, tower, device_ids, n_devices, dtype, max_batch, nullptr, out);
}

int clipgpu_create_ex(const char* model_dir, int tower, const int* device_ids, int n_devices, int dtype,
                      int max_batch, const clipgpu_options* opts_in, clipgpu_engine** out) {
  return guarded([&]() {
    if (!out) throw ClipErr(CLIPGPU_ERR_INVALID, "out is NULL");
    *out = nullptr;
    clipgpu_options opts;
    std::memset(&opts, 0, sizeof(opts));
    opts.struct_size = sizeof(opts);
    if (opts_in) {  // an older caller's smaller struct: its prefix, defaults for the rest
      // the sizes of the struct's published versions only: v2 (through `communicator`), v3 (through
      // `mx_layers`) and v4 (a size ending inside a field would copy part of it)
      if (opts_in->struct_size != offsetof(clipgpu_options, graphs) &&
          opts_in->struct_size != offsetof(clipgpu_options, residual) && opts_in->struct_size != sizeof(opts))
        throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.struct_size: call clipgpu_options_init first");
      std::memcpy(&opts, opts_in, opts_in->struct_size);
    }
    if (opts.mx_sites & ~(CLIPGPU_MX_QKV | CLIPGPU_MX_FC | CLIPGPU_MX_PROJ))
      throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.mx_sites: unknown bits");
    if (opts.lanes < 0 || opts.lanes > 4) throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.lanes must be 0..4");
    if (opts.tuning < 0 || opts.tuning > 2) throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.tuning must be 0, 1 or 2");
    for (int32_t v : {opts.graphs, opts.prune_last, opts.trim_text})
      if (v < -1 || v > 1) throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options graphs / prune_last / trim_text: -1, 0 or 1");
    for (int i = 0; i < 5; ++i) {
      const int t = i < 4 ? opts.gemm_tiles[i] : opts.patch_tile;
      if (t != 0 && t != -1 && !gemm_tile_built(t))
        throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.gemm_tiles / patch_tile: " + std::to_string(t) +
                                               " is not a GEMM tile this library builds");
    }
    if (opts.mx_layers != 0 && dtype != CLIPGPU_DTYPE_FP8)
      throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.mx_layers needs dtype CLIPGPU_DTYPE_FP8");
    if (opts.residual < 0 || opts.residual > CLIPGPU_RESIDUAL_F16)
      throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.residual must be 0, 1 (f32) or 2 (f16)");
    if (opts.ln_fold < -1 || opts.ln_fold > 1)
      throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.ln_fold must be -1, 0 or 1");
    if (opts.communicator < 0 || opts.communicator > 1)
      throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.communicator must be 0 or 1");
    if (!model_dir) throw ClipErr(CLIPGPU_ERR_INVALID, "model_dir is NULL");
    if (tower != CLIPGPU_TOWER_VISION && tower != CLIPGPU_TOWER_TEXT) throw ClipErr(CLIPGPU_ERR_INVALID, "bad tower");
    if (dtype != CLIPGPU_DTYPE_BF16 && dtype != CLIPGPU_DTYPE_F16 && dtype != CLIPGPU_DTYPE_FP8)
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad dtype");
    if (max_batch <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "max_batch must be > 0");
    const std::string dir(model_dir);
    struct stat st;
    if (::stat(dir.c_str(), &st) != 0 || !S_ISDIR(st.st_mode))
      throw ClipErr(CLIPGPU_ERR_CONFIG, "Model folder not found: '" + dir + "'");  // ClipError::ModelFolderNotFound
    for (const char* f : {"open_clip_config.json", "model_config.json"})
      if (!file_exists(dir + "/" + f))
        throw ClipErr(CLIPGPU_ERR_CONFIG, std::string("Missing model file '") + f + "' in folder '" + dir + "'");
    OpenClipConfig oc;
    try {
      oc = load_open_clip_config(dir + "/open_clip_config.json");
    } catch (const std::runtime_error& ex) {
      throw ClipErr(CLIPGPU_ERR_CONFIG, ex.what());
    }
    std::unique_ptr<clipgpu_engine> e(new clipgpu_engine());
    e->spec = tower == CLIPGPU_TOWER_VISION ? oc.vision : oc.text;
    e->pre = oc.pre;
    e->dt = dtype == CLIPGPU_DTYPE_F16 ? DT_F16 : DT_BF16;  // fp8 engines keep bf16 outside the MX GEMMs
    e->mx = dtype == CLIPGPU_DTYPE_FP8;
    if (e->mx) {  // the MX split: the options' bits, else all three sites
      const uint32_t bits = opts.mx_sites ? opts.mx_sites : (CLIPGPU_MX_QKV | CLIPGPU_MX_FC | CLIPGPU_MX_PROJ);
      e->mx_site[GS_QKV] = (bits & CLIPGPU_MX_QKV) != 0;
      e->mx_site[GS_FC] = (bits & CLIPGPU_MX_FC) != 0;
      e->mx_site[GS_PROJ] = (bits & CLIPGPU_MX_PROJ) != 0;
      if (e->mx_site[GS_PROJ] && !e->mx_site[GS_FC])
        throw ClipErr(CLIPGPU_ERR_INVALID, "MX sites: proj in MX needs fc in MX");
      if (e->spec.layers < 32 && (opts.mx_layers >> e->spec.layers) != 0)
        throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.mx_layers: bit set at or beyond the tower's " +
                                               std::to_string(e->spec.layers) + " layers");
      e->mx_layers = opts.mx_layers ? (uint64_t)opts.mx_layers : ~0ull;
    } else if (opts.mx_sites) {
      throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.mx_sites needs dtype CLIPGPU_DTYPE_FP8");
    }
    e->max_batch = max_batch;
    if (opts.lanes > 0) {
      e->lanes = opts.lanes;
      e->lanes_pinned = true;
    } else {
      e->lanes = 2;  // host-path staging slots (run_host_shard); the device-side lane count is the table's
    }
    e->tuning = opts.tuning;
    e->dev_lanes = e->lanes;
    e->graphs = opts.graphs != -1;
    e->prune = opts.prune_last != -1;
    e->trim = opts.trim_text != -1;
    {  // the residual stream's storage (clipgpu_options.residual; kResidualDefault when 0)
      const int res = opts.residual ? opts.residual : kResidualDefault;
      const bool f16_ok = e->spec.family != FAMILY_SIGLIP;
      if (opts.residual == CLIPGPU_RESIDUAL_F16 && !f16_ok)
        throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_options.residual = f16: CLIP-family engines only");
      e->x16 = res == CLIPGPU_RESIDUAL_F16 && f16_ok;
      // the LayerNorm fold (clipgpu_options.ln_fold): the f16 stream, a QuickGELU / GELU MLP
      const bool fold_ok = e->x16 && !e->mx && (e->spec.act == ACT_QUICK_GELU || e->spec.act == ACT_GELU);
      if (opts.ln_fold == 1 && !fold_ok)
        throw ClipErr(CLIPGPU_ERR_INVALID,
                      "clipgpu_options.ln_fold = 1: needs a bf16 / f16 engine, the f16 residual stream and a "
                      "QuickGELU / GELU MLP");
      e->lnf = fold_ok && opts.ln_fold != -1;
    }
    for (int i = 0; i < 4; ++i) e->pin_tiles[i] = opts.gemm_tiles[i];
    e->pin_patch = opts.patch_tile;
    const TowerSpec& s = e->spec;
    if (!s.unsupported.empty()) throw ClipErr(CLIPGPU_ERR_CONFIG, s.unsupported);
    if (s.heads <= 0 || s.width % s.heads || s.width % 64)
      throw ClipErr(CLIPGPU_ERR_CONFIG, "Configuration error: width must be a multiple of 64 and of heads");
    const int hd = s.width / s.heads;
    if (hd != 64 && hd != 72 && hd != 80)
      throw ClipErr(CLIPGPU_ERR_CONFIG, "Configuration error: head dim " + std::to_string(hd) + " not supported (64, 72, 80)");
    if (s.width > 1280) throw ClipErr(CLIPGPU_ERR_CONFIG, "Configuration error: width > 1280 not supported yet");
    if (e->mx && (s.width % 128 || mlp_pad(s) % 128))
      throw ClipErr(CLIPGPU_ERR_CONFIG, "Configuration error: the fp8 path needs width and MLP width % 128 == 0");
    if (s.tokens() > 1024) throw ClipErr(CLIPGPU_ERR_CONFIG, "Configuration error: > 1024 tokens not supported yet");
    if (s.tower == TOWER_VISION) {
      if (s.image_size % s.patch_size)
        throw ClipErr(CLIPGPU_ERR_CONFIG, "Configuration error: image_size must be a multiple of patch_size");
      e->in_bytes_per_row = (size_t)3 * s.image_size * s.image_size * 4;  // f32 (u8 path uses a quarter)
    } else {
      e->in_bytes_per_row = (size_t)s.context_length * 8;
    }
    // weights
    TensorMap m;
    try {
      m = load_tower_weights(dir, s);
    } catch (const std::runtime_error& ex) {
      throw ClipErr(CLIPGPU_ERR_CONFIG, ex.what());
    }
    int ndev = 0;
    HIP_CHECK(hipGetDeviceCount(&ndev));
    std::vector<int> devs;
    if (device_ids && n_devices > 0) devs.assign(device_ids, device_ids + n_devices);
    else devs.push_back(0);
    for (int d : devs)
      if (d < 0 || d >= ndev) throw ClipErr(CLIPGPU_ERR_DEVICE, "device id " + std::to_string(d) + " not available");
    e->reps.resize(devs.size());
    for (size_t i = 0; i < devs.size(); ++i) {
      Replica& r = e->reps[i];
      r.device = devs[i];
      HIP_CHECK(hipSetDevice(r.device));
      HIP_CHECK(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
      upload_weights(*e, r, m);
      alloc_workspace(*e, r);
      if (i == 0) {  // one tile choice, shared by identical devices
        if (e->tuning) {
          autotune_tiles(*e, r);
          apply_tile_pins(*e);
          tune_forward(*e, r);
        } else {
          table_tiles(*e);
          apply_tile_pins(*e);
        }
      }
    }
    // A multi-device handle over distinct devices gets one communicator (ncclCommInitAll; rank i
    // = device_ids[i]; RCCL refuses two ranks on one GPU, so a handle that lists a device twice
    // keeps the host-buffer sharding and has no collective entry points).  It is created on the
    // first gathered call (ensure_comm) unless the options ask for it now: creation and the
    // host-buffer entry points never depend on RCCL.  A one-device handle gets a one-rank clique
    // through the same code when clipgpu_options.communicator = 1 asks for one (else it joins a
    // deployment's communicator with clipgpu_comm_init_rank).
    bool distinct = devs.size() > 1 || (devs.size() == 1 && opts.communicator == 1);
    for (size_t i = 0; i < devs.size() && distinct; ++i)
      for (size_t j = i + 1; j < devs.size(); ++j) distinct = distinct && devs[i] != devs[j];
    if (distinct) {
      e->comm_devs = devs;
      e->comm_pending = true;
      e->comm_nranks = (int)devs.size();
      e->comm_rank0 = 0;
      if (opts.communicator == 1) ensure_comm(*e);
    }
    *out = e.release();
  });
}

void clipgpu_destroy(clipgpu_engine* e) {
  if (!e) return;
  for (hipEvent_t ev : e->prof.pool) (void)hipEventDestroy(ev);
  destroy_comms(*e);
  for (auto& r : e->reps) destroy_replica(r);
  delete e;
}

int clipgpu_embed_dim(const clipgpu_engine* e) { return e ? e->spec.embed_dim : -1; }
int clipgpu_input_size(const clipgpu_engine* e) {
  return e ? (e->spec.tower == TOWER_VISION ? e->spec.image_size : e->spec.context_length) : -1;
}
int clipgpu_num_devices(const clipgpu_engine* e) { return e ? (int)e->reps.size() : -1; }

static void need_tower(const clipgpu_engine* e, int tower) {
  if (!e) throw ClipErr(CLIPGPU_ERR_INVALID, "engine is NULL");
  if (e->spec.tower != tower)
    throw ClipErr(CLIPGPU_ERR_INVALID, tower == TOWER_VISION ? "engine is not a vision tower" : "engine is not a text tower");
}

int clipgpu_embed_pixels(clipgpu_engine* e, const float* nchw, int64_t B, int64_t S, float* out) {
  return guarded([&]() {
    need_tower(e, TOWER_VISION);
    if (B <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");
    if (!nchw || !out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    if (S != e->spec.image_size)
      throw ClipErr(CLIPGPU_ERR_INVALID, "Shape error: expected image size " + std::to_string(e->spec.image_size));
    std::lock_guard<std::mutex> lk(e->mu);
    run_host(*e, IN_F32, HostRows{(const char*)nchw, nullptr, (size_t)3 * S * S * 4}, B, nullptr, nullptr, out);
  });
}

int clipgpu_embed_u8(clipgpu_engine* e, const uint8_t* nhwc, int64_t B, int64_t S, const float mean[3],
                     const float stdv[3], float* out) {
  return guarded([&]() {
    need_tower(e, TOWER_VISION);
    if (B <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");
    if (!nhwc || !out || !mean || !stdv) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    if (S != e->spec.image_size)
      throw ClipErr(CLIPGPU_ERR_INVALID, "Shape error: expected image size " + std::to_string(e->spec.image_size));
    std::lock_guard<std::mutex> lk(e->mu);
    run_host(*e, IN_U8, HostRows{(const char*)nhwc, nullptr, (size_t)3 * S * S}, B, mean, stdv, out);
  });
}

int clipgpu_host_register(void* ptr, size_t bytes) {
  return guarded([&]() {
    if (!ptr || bytes == 0) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL / empty host range");
    HostRanges& h = host_ranges();
    std::lock_guard<std::mutex> lk(h.mu);
    const uintptr_t a = (uintptr_t)ptr;
    for (const auto& rg : h.r)
      if (a < rg.first + rg.second && rg.first < a + bytes)
        throw ClipErr(CLIPGPU_ERR_INVALID, "host range overlaps a registered one");
    // hipHostRegister pins whole pages: two ranges that share a page would pin it twice, and unregistering
    // one would unpin it under the other (and leave the runtime's page mapping stale for whatever the
    // allocator puts there next).  Such a range is refused; page-owning buffers (engine.py host_buffer)
    // never share one.
    const uintptr_t pg = (uintptr_t)kHostPage;
    for (const auto& rg : h.r)
      if (a / pg <= (rg.first + rg.second - 1) / pg && rg.first / pg <= (a + bytes - 1) / pg)
        throw ClipErr(CLIPGPU_ERR_INVALID,
                      "host range shares a memory page with a registered one (registration pins whole pages): "
                      "register page-aligned buffers");
    HIP_CHECK(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));  // every device
    h.r.emplace_back(a, bytes);
  });
}

int clipgpu_host_unregister(void* ptr) {
  return guarded([&]() {
    HostRanges& h = host_ranges();
    std::lock_guard<std::mutex> lk(h.mu);
    for (size_t i = 0; i < h.r.size(); ++i)
      if (h.r[i].first == (uintptr_t)ptr) {
        // no transfer of any device may still reference the range
        int ndev = 0;
        HIP_CHECK(hipGetDeviceCount(&ndev));
        int cur = 0;
        HIP_CHECK(hipGetDevice(&cur));
        for (int d = 0; d < ndev; ++d) {
          HIP_CHECK(hipSetDevice(d));
          HIP_CHECK(hipDeviceSynchronize());
        }
        HIP_CHECK(hipSetDevice(cur));
        HIP_CHECK(hipHostUnregister(ptr));
        h.r.erase(h.r.begin() + (long)i);
        return;
      }
    throw ClipErr(CLIPGPU_ERR_INVALID, "host range not registered");
  });
}

int clipgpu_embed_tokens(clipgpu_engine* e, const int64_t* ids, const int64_t* mask, int64_t B, int64_t T,
                         float* out) {
  (void)mask;
  return guarded([&]() {
    need_tower(e, TOWER_TEXT);
    if (B <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");
    if (!ids || !out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    if (T != e->spec.context_length)
      throw ClipErr(CLIPGPU_ERR_INVALID,
                    "Shape error: expected context length " + std::to_string(e->spec.context_length));
    for (int64_t i = 0; i < B * T; ++i)
      if (ids[i] < 0 || ids[i] >= e->spec.vocab_size)
        throw ClipErr(CLIPGPU_ERR_INVALID, "Inference error: token id " + std::to_string(ids[i]) + " out of range");
    // Sequence trimming: the pooled row of a sequence is its first argmax (EOT) token and
    // attention is causal, so tokens past the batch's last EOT never reach an embedding.
    // The batch runs on its first Tc = max(EOT index) + 1 tokens, rounded up to a multiple of 16,
    // bit-identical
    // (test_text_trim_is_bit_exact).  clipgpu_options.trim_text = -1 disables.  A trimmed batch is
    // a private copy, so it is staged even when `ids` lies in a registered range.
    int64_t Tc = T;
    // only for the causal, EOT-pooled (CLIP) form: SigLIP2's text tower attends to and pools
    // the last context position
    if (e->trim && e->spec.causal && !e->spec.pool_last) {
      Tc = 1;
      for (int64_t b = 0; b < B && Tc < T; ++b) {
        const int64_t* row = ids + b * T;
        int64_t best = 0;
        for (int64_t t = 1; t < T; ++t)
          if (row[t] > row[best]) best = t;
        Tc = std::max<int64_t>(Tc, best + 1);
      }
      // rounded up to a multiple of 16 (the causal key tiles are 16 wide, so any Tc past the
      // last EOT gives the same bits): at most ceil(T / 16) lengths reach the graph cache
      Tc = std::min<int64_t>(T, std::max<int64_t>((Tc + 15) / 16 * 16, 16));
    }
    std::vector<int64_t> trimmed;
    const int64_t* src = ids;
    if (Tc < T) {
      trimmed.resize((size_t)(B * Tc));
      for (int64_t b = 0; b < B; ++b) std::memcpy(&trimmed[(size_t)(b * Tc)], ids + b * T, (size_t)Tc * 8);
      src = trimmed.data();
    }
    std::lock_guard<std::mutex> lk(e->mu);
    run_host(*e, IN_IDS, HostRows{(const char*)src, nullptr, (size_t)Tc * 8}, B, nullptr, nullptr, out, (int)Tc);
  });
}

int clipgpu_embed_pixels_device(clipgpu_engine* e, const float* d_nchw, int64_t B, float* d_out, void* stream) {
  return guarded([&]() {
    need_tower(e, TOWER_VISION);
    if (B <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");
    if (B > e->max_batch) throw ClipErr(CLIPGPU_ERR_INVALID, "B exceeds max_batch");
    std::lock_guard<std::mutex> lk(e->mu);  // one enqueue per handle at a time (graph cache, workspace)
    Replica& r = e->reps[0];
    HIP_CHECK(hipSetDevice(r.device));
    run_graph(*e, r, {1, (uint64_t)d_nchw, (uint64_t)d_out, (uint64_t)B}, (hipStream_t)stream,
              [&](hipStream_t gs) { vision_forward_lanes(*e, r, d_nchw, A_IMG_F32, nullptr, nullptr, (int)B, d_out, gs); });
  });
}

int clipgpu_embed_u8_device(clipgpu_engine* e, const uint8_t* d_nhwc, int64_t B, const float mean[3],
                            const float stdv[3], float* d_out, void* stream) {
  return guarded([&]() {
    need_tower(e, TOWER_VISION);
    if (B <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");
    if (B > e->max_batch) throw ClipErr(CLIPGPU_ERR_INVALID, "B exceeds max_batch");
    if (!mean || !stdv) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL mean/std");
    std::lock_guard<std::mutex> lk(e->mu);  // one enqueue per handle at a time (graph cache, workspace)
    Replica& r = e->reps[0];
    HIP_CHECK(hipSetDevice(r.device));
    run_graph(*e, r,
              {2, (uint64_t)d_nhwc, (uint64_t)d_out, (uint64_t)B, fbits(mean, 0), fbits(mean, 1), fbits(mean, 2),
               fbits(stdv, 0), fbits(stdv, 1), fbits(stdv, 2)},
              (hipStream_t)stream,
              [&](hipStream_t gs) { vision_forward_lanes(*e, r, d_nhwc, A_IMG_U8, mean, stdv, (int)B, d_out, gs); });
  });
}

int clipgpu_embed_images_rgb8(clipgpu_engine* e, const uint8_t* const* images, const int* widths,
                              const int* heights, int64_t n, float* out) {
  return guarded([&]() {
    need_tower(e, TOWER_VISION);
    if (n <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");  // src/vision.rs:121-123
    if (!images || !widths || !heights || !out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    for (int64_t i = 0; i < n; ++i) {
      if (!images[i]) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL image");
      if (widths[i] <= 0 || heights[i] <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Resize error: empty image");
    }
    std::lock_guard<std::mutex> lk(e->mu);
    // A batch of S x S images needs no resize (the plan is the identity: a unit tap per output, exact) --
    // the images are the u8 NHWC rows, and the batch takes the u8 host path (copy pool staging in pieces,
    // copy-stream H2Ds, alternating buffer sets), bit-identical to the resize path
    // (test_embed_images_rgb8_identity_batches_take_the_u8_path).
    const int S = e->spec.image_size;
    bool identity = true;
    for (int64_t i = 0; i < n && identity; ++i) identity = widths[i] == S && heights[i] == S;
    if (identity) {
      const ResizePlan p = make_resize_plan(S, S, S, e->pre.interpolation, e->pre.resize_mode);
      identity = !p.need_h && !p.need_v;
    }
    if (identity && !e->rgb8_resize_always) {
      run_host(*e, IN_U8, HostRows{nullptr, (const void* const*)images, (size_t)3 * S * S}, n, e->pre.mean,
               e->pre.stdv, out);
      return;
    }
    run_sharded(*e, n, [&](Replica& r, int64_t b0, int64_t b1) {
      run_images_shard(*e, r, images, widths, heights, b0, b1, out);
    });
  });
}

static void check_similarity_args(int64_t n_img, int64_t n_txt, int64_t E, int activation, int axis) {
  if (n_img <= 0 || n_txt <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");
  if (E <= 0 || E % 16) throw ClipErr(CLIPGPU_ERR_INVALID, "Shape error: embedding dim must be a multiple of 16");
  if (n_img > (1L << 22) || n_txt > (1L << 30) || n_img * n_txt > (1L << 40))
    throw ClipErr(CLIPGPU_ERR_INVALID, "Shape error: similarity matrix too large");
  if (activation < CLIPGPU_SIM_SOFTMAX || activation > CLIPGPU_SIM_LOGITS || axis < 0 || axis > 1)
    throw ClipErr(CLIPGPU_ERR_INVALID, "bad activation / axis");
}

int clipgpu_similarity_device(const float* d_img, int64_t n_img, const float* d_txt, int64_t n_txt, int64_t E,
                              float logit_scale, float logit_bias, int activation, int axis, float* d_out,
                              void* stream) {
  return guarded([&]() {
    check_similarity_args(n_img, n_txt, E, activation, axis);
    if (!d_img || !d_txt || !d_out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    check(launch_similarity(d_img, (int)n_img, d_txt, (int)n_txt, (int)E, logit_scale, logit_bias, activation, axis,
                            d_out, (hipStream_t)stream),
          "similarity");
  });
}

int clipgpu_similarity(int device, const float* img, int64_t n_img, const float* txt, int64_t n_txt, int64_t E,
                       float logit_scale, float logit_bias, int activation, int axis, float* out) {
  return guarded([&]() {
    check_similarity_args(n_img, n_txt, E, activation, axis);
    if (!img || !txt || !out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    HIP_CHECK(hipSetDevice(device));
    const size_t bi = (size_t)n_img * E * 4, bt = (size_t)n_txt * E * 4, bo = (size_t)n_img * n_txt * 4;
    char* d = nullptr;
    HIP_CHECK(hipMalloc((void**)&d, align256(bi) + align256(bt) + bo));
    float *di = (float*)d, *dt = (float*)(d + align256(bi)), *dO = (float*)(d + align256(bi) + align256(bt));
    hipError_t err = copy_h2d(di, img, bi);
    if (err == hipSuccess) err = copy_h2d(dt, txt, bt);
    if (err == hipSuccess)
      err = launch_similarity(di, (int)n_img, dt, (int)n_txt, (int)E, logit_scale, logit_bias, activation, axis, dO,
                              nullptr);
    if (err == hipSuccess) err = copy_d2h(out, dO, bo);
    (void)hipFree(d);
    check(err, "similarity");
  });
}

int clipgpu_embed_tokens_device(clipgpu_engine* e, const int64_t* d_ids, int64_t B, float* d_out, void* stream) {
  return guarded([&]() {
    need_tower(e, TOWER_TEXT);
    if (B <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "Empty batch");
    if (B > e->max_batch) throw ClipErr(CLIPGPU_ERR_INVALID, "B exceeds max_batch");
    std::lock_guard<std::mutex> lk(e->mu);  // one enqueue per handle at a time (graph cache, workspace)
    Replica& r = e->reps[0];
    HIP_CHECK(hipSetDevice(r.device));
    run_graph(*e, r, {3, (uint64_t)d_ids, (uint64_t)d_out, (uint64_t)B}, (hipStream_t)stream,
              [&](hipStream_t gs) { text_forward_lanes(*e, r, d_ids, (int)B, d_out, gs); });
  });
}

int clipgpu_comm_unique_id(uint8_t* id) {
  return guarded([&]() {
    if (!id) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL id");
    ncclUniqueId u;
    NCCL_CHECK(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  });
}

int clipgpu_comm_init_rank(clipgpu_engine* e, const uint8_t* id, int nranks, int rank) {
  return guarded([&]() {
    if (!e || !id) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL argument");
    if (e->reps.size() != 1) throw ClipErr(CLIPGPU_ERR_INVALID, "clipgpu_comm_init_rank needs a one-device handle");
    if (nranks < 1 || rank < 0 || rank >= nranks) throw ClipErr(CLIPGPU_ERR_INVALID, "bad nranks / rank");
    std::lock_guard<std::mutex> lk(e->mu);
    Replica& r = e->reps[0];
    if (r.comm) throw ClipErr(CLIPGPU_ERR_INVALID, "the handle already has a communicator");
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    HIP_CHECK(hipSetDevice(r.device));
    NCCL_CHECK(ncclCommInitRank(&r.comm, nranks, u, rank));
    e->comm_nranks = nranks;
    e->comm_rank0 = rank;
  });
}

int clipgpu_comm_info(const clipgpu_engine* e, int* nranks, int* rank0) {
  return guarded([&]() {
    if (!e || !nranks || !rank0) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL argument");
    *nranks = e->comm_nranks;
    *rank0 = e->comm_rank0;
  });
}

int clipgpu_embed_pixels_gather_device(clipgpu_engine* e, const float* const* d_nchw, const int64_t* rows,
                                       float* const* d_out, void* const* streams) {
  return guarded([&]() {
    need_tower(e, TOWER_VISION);
    if (!d_nchw || !rows || !d_out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    std::lock_guard<std::mutex> lk(e->mu);
    const size_t row_bytes = (size_t)3 * e->spec.image_size * e->spec.image_size * 4;
    sharded_gather(*e, rows, d_out, streams, [&](Replica& r, int i, int64_t c0, int n, float* dst, hipStream_t st) {
      if (!d_nchw[i]) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
      const float* src = (const float*)((const char*)d_nchw[i] + c0 * row_bytes);
      run_graph(*e, r, {1, (uint64_t)src, (uint64_t)dst, (uint64_t)n}, st, [&](hipStream_t gs) {
        vision_forward_lanes(*e, r, src, A_IMG_F32, nullptr, nullptr, n, dst, gs);
      });
    });
  });
}

int clipgpu_embed_tokens_gather_device(clipgpu_engine* e, const int64_t* const* d_ids, const int64_t* rows,
                                       float* const* d_out, void* const* streams) {
  return guarded([&]() {
    need_tower(e, TOWER_TEXT);
    if (!d_ids || !rows || !d_out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    std::lock_guard<std::mutex> lk(e->mu);
    const int T = e->spec.context_length;
    sharded_gather(*e, rows, d_out, streams, [&](Replica& r, int i, int64_t c0, int n, float* dst, hipStream_t st) {
      if (!d_ids[i]) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
      const int64_t* src = d_ids[i] + c0 * T;
      run_graph(*e, r, {3, (uint64_t)src, (uint64_t)dst, (uint64_t)n}, st,
                [&](hipStream_t gs) { text_forward_lanes(*e, r, src, n, dst, gs); });
    });
  });
}

int clipgpu_test_resize_rgb8_gpu(const uint8_t* const* images, const int* widths, const int* heights, int64_t n,
                                 int size, const char* interpolation, const char* resize_mode, uint8_t* out) {
  return guarded([&]() {
    if (n <= 0 || n > 65535 || size <= 0) throw ClipErr(CLIPGPU_ERR_INVALID, "bad resize batch");
    const ResizeBatch b = plan_resize_batch(size, interpolation ? interpolation : "bicubic",
                                            resize_mode ? resize_mode : "shortest", widths, heights, 0, (int)n);
    const size_t desc_bytes = align16(b.d.size() * sizeof(ResizeImage));
    const size_t ints_bytes = align16(b.ints.size() * sizeof(int));
    std::vector<char> host(desc_bytes + ints_bytes + b.raw_bytes);
    std::memcpy(host.data(), b.d.data(), b.d.size() * sizeof(ResizeImage));
    std::memcpy(host.data() + desc_bytes, b.ints.data(), b.ints.size() * sizeof(int));
    for (int64_t i = 0; i < n; ++i)
    {
      std::vector<CopyTask> tasks;
      add_window_tasks(tasks, b, (int)i, host.data() + desc_bytes + ints_bytes + b.raw_off[i], images[i], widths[i]);
      pool_copy(tasks);
    }
    char* dev = nullptr;
    uint8_t *tmp = nullptr, *dout = nullptr;
    const size_t out_bytes = (size_t)n * size * size * 3;
    HIP_CHECK(hipMalloc((void**)&dev, host.size()));
    HIP_CHECK(hipMalloc((void**)&tmp, std::max<size_t>(b.tmp_bytes, 16)));
    HIP_CHECK(hipMalloc((void**)&dout, out_bytes));
    HIP_CHECK(copy_h2d(dev, host.data(), host.size()));
    const hipError_t err = launch_resize((const uint8_t*)dev + desc_bytes + ints_bytes, tmp,
                                         (const int*)(dev + desc_bytes), (const ResizeImage*)dev, (int)n, b.max_th,
                                         size, dout, nullptr);
    const hipError_t err2 = copy_d2h(out, dout, out_bytes);
    (void)hipFree(dev);
    (void)hipFree(tmp);
    (void)hipFree(dout);
    check(err, "resize");
    check(err2, "resize copy-out");
  });
}

int clipgpu_test_read_weights(const char* model_dir, int tower, const char* name, float* out, int64_t n) {
  return guarded([&]() {
    if (!model_dir || !name || !out) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL argument");
    if (tower != CLIPGPU_TOWER_VISION && tower != CLIPGPU_TOWER_TEXT) throw ClipErr(CLIPGPU_ERR_INVALID, "bad tower");
    const std::string dir(model_dir);
    TensorMap m;
    try {
      const OpenClipConfig oc = load_open_clip_config(dir + "/open_clip_config.json");
      m = load_tower_weights(dir, tower == CLIPGPU_TOWER_VISION ? oc.vision : oc.text);
    } catch (const std::runtime_error& ex) {
      throw ClipErr(CLIPGPU_ERR_CONFIG, ex.what());
    }
    auto it = m.find(name);
    if (it == m.end()) throw ClipErr(CLIPGPU_ERR_INVALID, std::string("no parameter ") + name);
    if (it->second.numel() != n) throw ClipErr(CLIPGPU_ERR_INVALID, "size mismatch for " + std::string(name));
    std::memcpy(out, it->second.data.data(), (size_t)n * sizeof(float));
  });
}

int clipgpu_test_engine_tiles(const clipgpu_engine* e, int tiles[4]) {
  return guarded([&]() {
    if (!e || !tiles) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL argument");
    for (int i = 0; i < 4; ++i) tiles[i] = e->mx_site[i] ? e->mxtile[i] : e->tile[i];
  });
}

int clipgpu_engine_info(const clipgpu_engine* e, int tiles[4], int* lanes, uint32_t* mx_sites) {
  return guarded([&]() {
    if (!e) throw ClipErr(CLIPGPU_ERR_INVALID, "engine is NULL");
    if (tiles)
      for (int i = 0; i < 4; ++i) tiles[i] = e->mx_site[i] ? e->mxtile[i] : e->tile[i];
    if (lanes) *lanes = e->dev_lanes;
    if (mx_sites)
      *mx_sites = (e->mx_site[GS_QKV] ? CLIPGPU_MX_QKV : 0u) | (e->mx_site[GS_FC] ? CLIPGPU_MX_FC : 0u) |
                  (e->mx_site[GS_PROJ] ? CLIPGPU_MX_PROJ : 0u);
  });
}

int clipgpu_test_force_broadcast(clipgpu_engine* e, int on) {
  return guarded([&]() {
    if (!e) throw ClipErr(CLIPGPU_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    e->force_bcast = on != 0;
  });
}

// A handle without a communicator takes the multi-device handle's lazy path: its own clique over its
// replicas' (distinct) devices, created by ensure_comm on the first gathered call.
int clipgpu_test_comm_lazy(clipgpu_engine* e) {
  return guarded([&]() {
    if (!e) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL handle");
    if (e->comm_nranks > 0) throw ClipErr(CLIPGPU_ERR_INVALID, "the handle already has a communicator");
    std::vector<int> devs;
    for (auto& r : e->reps) {
      for (int d : devs)
        if (d == r.device) throw ClipErr(CLIPGPU_ERR_INVALID, "a device listed twice has no clique");
      devs.push_back(r.device);
    }
    e->comm_devs = devs;
    e->comm_pending = true;
    e->comm_nranks = (int)devs.size();
    e->comm_rank0 = 0;
  });
}

int clipgpu_test_gather_plan(int nranks, const int64_t* rows, int64_t* off, int* equal) {
  return guarded([&]() {
    if (nranks < 1 || !rows || !off || !equal) throw ClipErr(CLIPGPU_ERR_INVALID, "bad arguments");
    const GatherPlan g = plan_gather(nranks, rows);
    for (int r = 0; r <= nranks; ++r) off[r] = g.off[r];
    *equal = g.equal ? 1 : 0;
  });
}

int clipgpu_test_host_plan(clipgpu_engine* e, int n_chunks, const int* bounds, int copy_stream) {
  return guarded([&]() {
    if (!e) throw ClipErr(CLIPGPU_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    // (copy_stream: the schedule variants of rounds 3-5 were removed in round 6; 0 and 1 both mean the one
    // schedule run_host_shard has)
    if (copy_stream != 0 && copy_stream != 1) throw ClipErr(CLIPGPU_ERR_INVALID, "copy_stream: 0 or 1");
    e->host_part.clear();
    if (n_chunks == 0) return;
    if (n_chunks < 1 || n_chunks > 4 || !bounds) throw ClipErr(CLIPGPU_ERR_INVALID, "1..4 chunks");
    std::vector<int> part{0};
    for (int i = 0; i < n_chunks - 1; ++i) {
      if (bounds[i] <= part.back() || bounds[i] >= e->max_batch)
        throw ClipErr(CLIPGPU_ERR_INVALID, "chunk bounds must increase inside (0, max_batch)");
      part.push_back(bounds[i]);
    }
    part.push_back(e->max_batch);
    e->host_part = part;
  });
}

int clipgpu_test_rgb8_resize_always(clipgpu_engine* e, int on) {
  return guarded([&]() {
    if (!e) throw ClipErr(CLIPGPU_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    e->rgb8_resize_always = on != 0;
  });
}

int clipgpu_test_engine_lanes(const clipgpu_engine* e, int* dev_lanes) {
  return guarded([&]() {
    if (!e || !dev_lanes) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL argument");
    *dev_lanes = e->dev_lanes;
  });
}

int clipgpu_test_engine_residual(const clipgpu_engine* e, int* residual, int* ln_fold) {
  return guarded([&]() {
    if (!e || !residual) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL argument");
    *residual = e->x16 ? CLIPGPU_RESIDUAL_F16 : CLIPGPU_RESIDUAL_F32;
    if (ln_fold) *ln_fold = e->lnf ? 1 : 0;
  });
}

int clipgpu_profile_enable(clipgpu_engine* e, unsigned mask) {
  return guarded([&]() {
    if (!e) throw ClipErr(CLIPGPU_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    Profiler& p = e->prof;
    for (auto& rec : p.pending) { (void)hipEventSynchronize(rec.b); }
    p.pending.clear();
    p.used = 0;
    for (int i = 0; i < PC_N; ++i) { p.total_ms[i] = 0; p.count[i] = 0; }
    p.mask = mask;
  });
}

int clipgpu_profile_read(clipgpu_engine* e, int category, double* total_ms, int64_t* launches) {
  return guarded([&]() {
    if (!e || category < 0 || category >= PC_N) throw ClipErr(CLIPGPU_ERR_INVALID, "bad profile query");
    std::lock_guard<std::mutex> lk(e->mu);
    Profiler& p = e->prof;
    for (auto& rec : p.pending) {
      HIP_CHECK(hipEventSynchronize(rec.b));
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, rec.a, rec.b));
      p.total_ms[rec.cat] += ms;
      p.count[rec.cat] += 1;
    }
    p.pending.clear();
    p.used = 0;
    if (total_ms) *total_ms = p.total_ms[category];
    if (launches) *launches = p.count[category];
  });
}

// The recorded launches as a timeline (tools/timeline.py): start / end of each in ms from the first
// recorded start, its category and lane (index of the lane stream it ran on, -1 for another stream).
// Consumes the records like clipgpu_profile_read (which then sees them in its totals).
int clipgpu_test_profile_timeline(clipgpu_engine* e, int64_t n_max, double* t0, double* t1, int* cat, int* lane,
                                  int64_t* n_out) {
  return guarded([&]() {
    if (!e || !n_out || n_max < 0 || (n_max > 0 && (!t0 || !t1 || !cat || !lane)))
      throw ClipErr(CLIPGPU_ERR_INVALID, "bad timeline query");
    std::lock_guard<std::mutex> lk(e->mu);
    Profiler& p = e->prof;
    int64_t n = 0;
    for (auto& rec : p.pending) HIP_CHECK(hipEventSynchronize(rec.b));
    for (auto& rec : p.pending) {
      float ms = 0.f, s0 = 0.f, s1 = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, rec.a, rec.b));
      p.total_ms[rec.cat] += ms;
      p.count[rec.cat] += 1;
      if (n < n_max) {
        HIP_CHECK(hipEventElapsedTime(&s0, p.pending[0].a, rec.a));
        HIP_CHECK(hipEventElapsedTime(&s1, p.pending[0].a, rec.b));
        t0[n] = s0;
        t1[n] = s1;
        cat[n] = rec.cat;
        int ln = -1;
        for (int i = 0; i < 4 && !e->reps.empty(); ++i)
          if (rec.st != nullptr && rec.st == e->reps[0].lane[i]) ln = i;
        lane[n] = ln;
      }
      ++n;
    }
    p.pending.clear();
    p.used = 0;
    *n_out = n;
  });
}

const char* clipgpu_profile_category_name(int category) {
  return (category >= 0 && category < PC_N) ? kProfNames[category] : "";
}

int clipgpu_synth_tensor(uint64_t seed, const char* name, double std_, double offset, float* out, int64_t n) {
  return guarded([&]() {
    if (!name || !out || n < 0) throw ClipErr(CLIPGPU_ERR_INVALID, "bad arguments");
    synth_fill(seed, name, std_, offset, out, n);
  });
}

}  // extern "C"
