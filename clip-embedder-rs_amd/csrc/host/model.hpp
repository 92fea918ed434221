// Host-side model description: configs from the model dir, tower specs, and
// host weight sources (seeded synthetic generator, open_clip safetensors).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace clipgpu {

// src/config.rs:49-64 (PreprocessCfg, defaults "bicubic" / "shortest").
struct PreprocessCfg {
  float mean[3] = {0.48145466f, 0.4578275f, 0.40821073f};
  float stdv[3] = {0.26862954f, 0.26130258f, 0.27577711f};
  std::string interpolation = "bicubic";
  std::string resize_mode = "shortest";
};

// src/config.rs:6-14 (ModelConfig), written by pull_onnx.py:128-150.
struct ModelConfig {
  bool tokenizer_needs_lowercase = false;
  std::string activation_function;  // empty == None
  bool has_logit_scale = false, has_logit_bias = false;
  float logit_scale = 1.0f, logit_bias = 0.0f;
  long pad_id = -1;  // -1 == None
};

enum Tower { TOWER_VISION = 0, TOWER_TEXT = 1 };
enum Family { FAMILY_CLIP = 0, FAMILY_SIGLIP = 1 };

// Architecture of one tower.  The reference never parses most of these
// (src/config.rs:36-47) because they are baked into the ONNX graphs; we derive
// them from open_clip's model_cfg with open_clip's defaults.
struct TowerSpec {
  int tower = TOWER_VISION;
  int width = 0, layers = 0, heads = 0, mlp_width = 0, embed_dim = 0;
  int act = 1;          // Act enum (common.hpp)
  float ln_eps = 1e-5f;
  // vision
  int image_size = 0, patch_size = 0;
  // FAMILY_CLIP: open_clip VisionTransformer (CLS token, ln_pre, CLS pooling, proj).
  // FAMILY_SIGLIP: timm ViT trunk of open_clip TimmModel (no CLS, no pre-norm, patch-conv
  // bias, final norm, MAP attention-pool head, timm_proj "none"; names visual.trunk.*).
  int family = 0;
  bool cls() const { return family == 0; }
  int grid() const { return patch_size ? image_size / patch_size : 0; }
  int tokens() const { return tower == TOWER_VISION ? grid() * grid() + (cls() ? 1 : 0) : context_length; }
  // text
  int context_length = 0, vocab_size = 0;
  // open_clip TextTransformer form: CLIP (causal mask, argmax / EOT pooling, projection matrix) or
  // SigLIP2 (text_cfg no_causal_mask, pool_type "last": the final context position, proj_bias:
  // text_projection is an nn.Linear with bias)
  bool causal = true, pool_last = false, proj_bias = false;
  // Non-empty: the config asks for a tower form the engine does not build (clipgpu_create fails
  // with this message; the other tower of the same folder still loads).
  std::string unsupported;
};

struct OpenClipConfig {
  int embed_dim = 0;
  TowerSpec vision, text;
  PreprocessCfg pre;
};

OpenClipConfig load_open_clip_config(const std::string& path);  // throws std::runtime_error
ModelConfig load_model_config(const std::string& path);

struct HostTensor {
  std::vector<int64_t> shape;
  std::vector<float> data;
  int64_t numel() const {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    return n;
  }
};
typedef std::map<std::string, HostTensor> TensorMap;

// Parameter inventory (open_clip state-dict names) of one tower: name, shape,
// init std, offset.  Mirrors oracle/weights.py exactly.
struct ParamDesc {
  std::string name;
  std::vector<int64_t> shape;
  double std;
  double offset;
};
std::vector<ParamDesc> tower_params(const TowerSpec& spec);

// splitmix64 counter generator (oracle/weights.py).
uint64_t fnv1a64(const std::string& s);
uint64_t mix64(uint64_t z);
void synth_fill(uint64_t seed, const std::string& name, double std, double offset, float* out, int64_t n);
TensorMap synth_weights(const TowerSpec& spec, uint64_t seed);

// open_clip_model.safetensors (F32 / F16 / BF16) -> f32 host tensors of one tower.
TensorMap load_safetensors(const std::string& path, const TowerSpec& spec);

// visual.onnx / text.onnx initializers (+ external .onnx.data), the reference's model
// folder layout (src/model_manager.rs:8-18) -> f32 host tensors of one tower.
TensorMap load_onnx(const std::string& path, const TowerSpec& spec);

// The weight source of a model folder, in order: open_clip_model.safetensors,
// visual.onnx / text.onnx, clipgpu_synthetic.json {"seed": N}.  Throws runtime_error.
TensorMap load_tower_weights(const std::string& dir, const TowerSpec& spec);

}  // namespace clipgpu
