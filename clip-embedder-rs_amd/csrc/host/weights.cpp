// Host weight sources.
//
//  * synth_*: the seeded splitmix64 counter generator shared with
//    oracle/weights.py (bit-exact; compiled with -ffp-contract=off).  Used for
//    synthetic-weight parity tests and benchmarks (no checkpoint can be fetched).
//  * load_safetensors: open_clip checkpoints (open_clip_model.safetensors, the
//    file open_clip's hf-hub loader reads — pull_onnx.py:98-102 loads the same
//    state dict before exporting the ONNX graphs).  ONNX initializer ingestion
//    (visual.onnx.data / text.onnx.data, src/model_manager.rs:8-18) is the next
//    row of SURVEY.md §8(f).
#include <cmath>
#include <cstring>
#include <fcntl.h>
#include <stdexcept>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "json.hpp"
#include "model.hpp"

namespace clipgpu {

uint64_t fnv1a64(const std::string& s) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 0x100000001B3ull;
  }
  return h;
}

uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void synth_fill(uint64_t seed, const std::string& name, double std_, double offset, float* out, int64_t n) {
  const uint64_t ts = mix64(seed ^ fnv1a64(name));
  const float amp = (float)(std_ * std::sqrt(3.0));
  const float off = (float)offset;
  const float k = 1.0f / 8388608.0f;  // 2^-23
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t z = mix64(ts + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull);
    const float u = (float)(z >> 40) * k - 1.0f;  // exact
    const float t = u * amp;                      // one rounding
    out[i] = t + off;                             // one rounding
  }
}

static const double LN_GAIN_STD = 0.1 / std::sqrt(3.0);
static const double LN_BIAS_STD = 0.05 / std::sqrt(3.0);
static const double LIN_BIAS_STD = 0.02 / std::sqrt(3.0);

static void block_params(std::vector<ParamDesc>& out, const std::string& pre, int64_t D, int64_t M, int64_t L) {
  const double attn_std = std::pow((double)D, -0.5);
  const double proj_std = std::pow((double)D, -0.5) * std::pow((double)(2 * L), -0.5);
  const double fc_std = std::pow((double)(2 * D), -0.5);
  out.push_back({pre + "ln_1.weight", {D}, LN_GAIN_STD, 1.0});
  out.push_back({pre + "ln_1.bias", {D}, LN_BIAS_STD, 0.0});
  out.push_back({pre + "attn.in_proj_weight", {3 * D, D}, attn_std, 0.0});
  out.push_back({pre + "attn.in_proj_bias", {3 * D}, LIN_BIAS_STD, 0.0});
  out.push_back({pre + "attn.out_proj.weight", {D, D}, proj_std, 0.0});
  out.push_back({pre + "attn.out_proj.bias", {D}, LIN_BIAS_STD, 0.0});
  out.push_back({pre + "ln_2.weight", {D}, LN_GAIN_STD, 1.0});
  out.push_back({pre + "ln_2.bias", {D}, LN_BIAS_STD, 0.0});
  out.push_back({pre + "mlp.c_fc.weight", {M, D}, fc_std, 0.0});
  out.push_back({pre + "mlp.c_fc.bias", {M}, LIN_BIAS_STD, 0.0});
  out.push_back({pre + "mlp.c_proj.weight", {D, M}, proj_std, 0.0});
  out.push_back({pre + "mlp.c_proj.bias", {D}, LIN_BIAS_STD, 0.0});
}

static void timm_block_params(std::vector<ParamDesc>& out, const std::string& pre, int64_t D, int64_t M, int64_t L) {
  const double attn_std = std::pow((double)D, -0.5);
  const double proj_std = std::pow((double)D, -0.5) * std::pow((double)(2 * L), -0.5);
  const double fc_std = std::pow((double)(2 * D), -0.5);
  out.push_back({pre + "norm1.weight", {D}, LN_GAIN_STD, 1.0});
  out.push_back({pre + "norm1.bias", {D}, LN_BIAS_STD, 0.0});
  out.push_back({pre + "attn.qkv.weight", {3 * D, D}, attn_std, 0.0});
  out.push_back({pre + "attn.qkv.bias", {3 * D}, LIN_BIAS_STD, 0.0});
  out.push_back({pre + "attn.proj.weight", {D, D}, proj_std, 0.0});
  out.push_back({pre + "attn.proj.bias", {D}, LIN_BIAS_STD, 0.0});
  out.push_back({pre + "norm2.weight", {D}, LN_GAIN_STD, 1.0});
  out.push_back({pre + "norm2.bias", {D}, LN_BIAS_STD, 0.0});
  out.push_back({pre + "mlp.fc1.weight", {M, D}, fc_std, 0.0});
  out.push_back({pre + "mlp.fc1.bias", {M}, LIN_BIAS_STD, 0.0});
  out.push_back({pre + "mlp.fc2.weight", {D, M}, proj_std, 0.0});
  out.push_back({pre + "mlp.fc2.bias", {D}, LIN_BIAS_STD, 0.0});
}

// open_clip TimmModel over a timm SigLIP ViT (oracle/weights.py siglip_vision_param_list).
static std::vector<ParamDesc> siglip_vision_params(const TowerSpec& s) {
  std::vector<ParamDesc> out;
  const int64_t D = s.width, L = s.layers, M = s.mlp_width, p = s.patch_size, G = s.grid();
  const double rD = std::pow((double)D, -0.5);
  const std::string t = "visual.trunk.", a = "visual.trunk.attn_pool.";
  out.push_back({t + "patch_embed.proj.weight", {D, 3, p, p}, std::pow((double)(3 * p * p), -0.5), 0.0});
  out.push_back({t + "patch_embed.proj.bias", {D}, LIN_BIAS_STD, 0.0});
  out.push_back({t + "pos_embed", {1, G * G, D}, rD, 0.0});
  for (int i = 0; i < L; ++i) timm_block_params(out, t + "blocks." + std::to_string(i) + ".", D, M, L);
  out.push_back({t + "norm.weight", {D}, LN_GAIN_STD, 1.0});
  out.push_back({t + "norm.bias", {D}, LN_BIAS_STD, 0.0});
  out.push_back({a + "latent", {1, 1, D}, rD, 0.0});
  out.push_back({a + "q.weight", {D, D}, rD, 0.0});
  out.push_back({a + "q.bias", {D}, LIN_BIAS_STD, 0.0});
  out.push_back({a + "kv.weight", {2 * D, D}, rD, 0.0});
  out.push_back({a + "kv.bias", {2 * D}, LIN_BIAS_STD, 0.0});
  out.push_back({a + "proj.weight", {D, D}, rD, 0.0});
  out.push_back({a + "proj.bias", {D}, LIN_BIAS_STD, 0.0});
  out.push_back({a + "norm.weight", {D}, LN_GAIN_STD, 1.0});
  out.push_back({a + "norm.bias", {D}, LN_BIAS_STD, 0.0});
  out.push_back({a + "mlp.fc1.weight", {M, D}, std::pow((double)(2 * D), -0.5), 0.0});
  out.push_back({a + "mlp.fc1.bias", {M}, LIN_BIAS_STD, 0.0});
  out.push_back({a + "mlp.fc2.weight", {D, M}, rD, 0.0});
  out.push_back({a + "mlp.fc2.bias", {D}, LIN_BIAS_STD, 0.0});
  return out;
}

std::vector<ParamDesc> tower_params(const TowerSpec& s) {
  if (s.tower == TOWER_VISION && s.family == FAMILY_SIGLIP) return siglip_vision_params(s);
  std::vector<ParamDesc> out;
  const int64_t D = s.width, L = s.layers, M = s.mlp_width, E = s.embed_dim;
  if (s.tower == TOWER_VISION) {
    const int64_t p = s.patch_size;
    out.push_back({"visual.conv1.weight", {D, 3, p, p}, std::pow((double)(3 * p * p), -0.5), 0.0});
    out.push_back({"visual.class_embedding", {D}, std::pow((double)D, -0.5), 0.0});
    out.push_back({"visual.positional_embedding", {(int64_t)s.tokens(), D}, std::pow((double)D, -0.5), 0.0});
    out.push_back({"visual.ln_pre.weight", {D}, LN_GAIN_STD, 1.0});
    out.push_back({"visual.ln_pre.bias", {D}, LN_BIAS_STD, 0.0});
    for (int i = 0; i < L; ++i)
      block_params(out, "visual.transformer.resblocks." + std::to_string(i) + ".", D, M, L);
    out.push_back({"visual.ln_post.weight", {D}, LN_GAIN_STD, 1.0});
    out.push_back({"visual.ln_post.bias", {D}, LN_BIAS_STD, 0.0});
    out.push_back({"visual.proj", {D, E}, std::pow((double)D, -0.5), 0.0});
  } else {
    out.push_back({"token_embedding.weight", {(int64_t)s.vocab_size, D}, 0.02, 0.0});
    out.push_back({"positional_embedding", {(int64_t)s.context_length, D}, 0.01, 0.0});
    for (int i = 0; i < L; ++i) block_params(out, "transformer.resblocks." + std::to_string(i) + ".", D, M, L);
    out.push_back({"ln_final.weight", {D}, LN_GAIN_STD, 1.0});
    out.push_back({"ln_final.bias", {D}, LN_BIAS_STD, 0.0});
    if (s.proj_bias) {  // open_clip nn.Linear(width, embed_dim)
      out.push_back({"text_projection.weight", {E, D}, std::pow((double)D, -0.5), 0.0});
      out.push_back({"text_projection.bias", {E}, 0.02, 0.0});
    } else {
      out.push_back({"text_projection", {D, E}, std::pow((double)D, -0.5), 0.0});
    }
  }
  return out;
}

TensorMap synth_weights(const TowerSpec& spec, uint64_t seed) {
  TensorMap m;
  for (const ParamDesc& p : tower_params(spec)) {
    HostTensor t;
    t.shape = p.shape;
    t.data.resize((size_t)t.numel());
    synth_fill(seed, p.name, p.std, p.offset, t.data.data(), t.numel());
    m.emplace(p.name, std::move(t));
  }
  return m;
}

float half_to_float(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000) << 16;
  uint32_t exp = (h >> 10) & 0x1F, man = h & 0x3FF;
  uint32_t bits;
  if (exp == 0) {
    if (man == 0) {
      bits = sign;
    } else {  // subnormal
      exp = 127 - 15 + 1;
      while (!(man & 0x400)) { man <<= 1; --exp; }
      man &= 0x3FF;
      bits = sign | (exp << 23) | (man << 13);
    }
  } else if (exp == 31) {
    bits = sign | 0x7F800000u | (man << 13);
  } else {
    bits = sign | ((exp - 15 + 127) << 23) | (man << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

TensorMap load_safetensors(const std::string& path, const TowerSpec& spec) {
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("IO error: cannot open '" + path + "'");
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < 8) {
    ::close(fd);
    throw std::runtime_error("Configuration error: '" + path + "' is not a safetensors file");
  }
  const size_t size = (size_t)st.st_size;
  void* map = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (map == MAP_FAILED) throw std::runtime_error("IO error: mmap failed for '" + path + "'");
  const unsigned char* base = (const unsigned char*)map;
  TensorMap out;
  try {
    uint64_t hlen = 0;
    std::memcpy(&hlen, base, 8);
    if (8 + hlen > size) throw std::runtime_error("Configuration error: truncated safetensors header");
    json::ValuePtr hdr = json::parse(std::string((const char*)base + 8, (size_t)hlen));
    const unsigned char* data = base + 8 + hlen;
    const size_t data_len = size - 8 - hlen;
    for (const ParamDesc& p : tower_params(spec)) {
      const json::Value* e = hdr->get(p.name);
      if (!e) throw std::runtime_error("Configuration error: tensor '" + p.name + "' missing from " + path);
      const std::string dt = e->get("dtype") ? e->get("dtype")->as_str("") : "";
      const json::Value* shp = e->get("shape");
      const json::Value* off = e->get("data_offsets");
      if (!shp || !off || off->arr.size() != 2) throw std::runtime_error("Configuration error: bad entry " + p.name);
      HostTensor t;
      for (auto& d : shp->arr) t.shape.push_back((int64_t)d->as_num(0));
      if (t.shape != p.shape) throw std::runtime_error("Shape error: '" + p.name + "' has an unexpected shape");
      const size_t s0 = (size_t)off->arr[0]->as_num(0), s1 = (size_t)off->arr[1]->as_num(0);
      const int64_t n = t.numel();
      const size_t esz = dt == "F32" ? 4 : (dt == "F16" || dt == "BF16") ? 2 : 0;
      if (!esz) throw std::runtime_error("Configuration error: unsupported dtype " + dt + " for " + p.name);
      if (s1 < s0 || s1 > data_len || (s1 - s0) != (size_t)n * esz)
        throw std::runtime_error("Configuration error: bad data_offsets for " + p.name);
      t.data.resize((size_t)n);
      const unsigned char* src = data + s0;
      for (int64_t i = 0; i < n; ++i) {
        if (dt == "F32") {
          std::memcpy(&t.data[i], src + 4 * i, 4);
        } else if (dt == "BF16") {
          uint16_t h;
          std::memcpy(&h, src + 2 * i, 2);
          uint32_t bits = (uint32_t)h << 16;
          std::memcpy(&t.data[i], &bits, 4);
        } else {
          uint16_t h;
          std::memcpy(&h, src + 2 * i, 2);
          t.data[i] = half_to_float(h);
        }
      }
      out.emplace(p.name, std::move(t));
    }
  } catch (...) {
    munmap(map, size);
    throw;
  }
  munmap(map, size);
  return out;
}

static bool is_file(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

TensorMap load_tower_weights(const std::string& dir, const TowerSpec& spec) {
  const std::string st_path = dir + "/open_clip_model.safetensors";
  const std::string onnx_name = spec.tower == TOWER_VISION ? "visual.onnx" : "text.onnx";
  const std::string syn_path = dir + "/clipgpu_synthetic.json";
  if (is_file(st_path)) return load_safetensors(st_path, spec);
  if (is_file(dir + "/" + onnx_name)) return load_onnx(dir + "/" + onnx_name, spec);  // pull_onnx.py export
  if (is_file(syn_path)) {
    json::ValuePtr j = json::parse_file(syn_path);
    const json::Value* sd = j->get("seed");
    if (!sd) throw std::runtime_error("Configuration error: clipgpu_synthetic.json has no seed");
    return synth_weights(spec, (uint64_t)sd->as_num(0));
  }
  throw std::runtime_error("Missing model file '" + onnx_name + "' in folder '" + dir + "'");
}

}  // namespace clipgpu
