// Config parsing for the model dir (src/config.rs restated in C++) plus the
// architecture fields the reference leaves inside the ONNX graphs.
#include <cmath>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "json.hpp"
#include "model.hpp"

namespace clipgpu {

namespace json {
ValuePtr parse_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("IO error: cannot open '" + path + "'");
  std::stringstream ss;
  ss << f.rdbuf();
  return parse(ss.str());
}
}  // namespace json

static int act_from(const json::Value& model_cfg, const json::Value* sub) {
  if (sub) {
    const json::Value* a = sub->get("act_layer");
    if (a && (a->as_str("") == "gelu_tanh" || a->as_str("") == "gelu_pytorch_tanh")) return 3;
    const json::Value* k = sub->get("act_kwargs");  // open_clip nn.GELU(approximate="tanh")
    if (k && k->get("approximate") && k->get("approximate")->as_str("") == "tanh") return 3;
  }
  const json::Value* q = model_cfg.get("quick_gelu");
  return (q && q->as_bool(false)) ? 1 : 2;  // ACT_QUICK_GELU : ACT_GELU
}

static int geti(const json::Value* o, const char* k, int dflt);

// timm SigLIP ViTs as open_clip TimmModel builds them (timm_model_name -> patch, width,
// depth, heads, mlp hidden): global_pool "map", GELU(tanh), LayerNorm eps 1e-6, no class
// token, no pre-norm, patch-embedding conv with bias (oracle/model_spec.py TIMM_SIGLIP).
static void timm_siglip_spec(const std::string& name, const json::Value* v, TowerSpec& vs) {
  struct Row { const char* prefix; int patch, width, layers, heads, mlp; };
  static const Row rows[] = {
      {"vit_base_patch16_siglip_", 16, 768, 12, 12, 3072},     {"vit_large_patch16_siglip_", 16, 1024, 24, 16, 4096},
      {"vit_so400m_patch14_siglip_", 14, 1152, 27, 16, 4304},  {"vit_so400m_patch16_siglip_", 16, 1152, 27, 16, 4304},
      {"vit_giantopt_patch16_siglip_", 16, 1536, 40, 16, 6144},
  };
  const Row* hit = nullptr;
  for (const Row& r : rows)
    if (name.rfind(r.prefix, 0) == 0) hit = &r;
  if (!hit) throw std::runtime_error("Configuration error: timm model '" + name + "' is not supported");
  const json::Value* pool = v->get("timm_pool");
  const json::Value* proj = v->get("timm_proj");
  if ((pool && !pool->is_null() && pool->as_str("") != "map") ||
      (proj && !proj->is_null() && proj->as_str("") != "none"))
    throw std::runtime_error("Configuration error: only timm_pool 'map' with timm_proj 'none' is supported");
  const json::Value* d = v->get("clipgpu_dims");  // synthetic test configs only: explicit (reduced) dims
  vs.family = FAMILY_SIGLIP;
  vs.patch_size = geti(d, "patch_size", hit->patch);
  vs.width = geti(d, "width", hit->width);
  vs.layers = geti(d, "layers", hit->layers);
  vs.heads = geti(d, "heads", hit->heads);
  vs.mlp_width = geti(d, "mlp_width", hit->mlp);
  vs.act = 3;  // ACT_GELU_TANH
  vs.ln_eps = 1e-6f;
}

static int geti(const json::Value* o, const char* k, int dflt) {
  const json::Value* v = o ? o->get(k) : nullptr;
  return v ? (int)v->as_num(dflt) : dflt;
}
static double getd(const json::Value* o, const char* k, double dflt) {
  const json::Value* v = o ? o->get(k) : nullptr;
  return v ? v->as_num(dflt) : dflt;
}

OpenClipConfig load_open_clip_config(const std::string& path) {
  json::ValuePtr root = json::parse_file(path);
  const json::Value* mc = root->get("model_cfg");
  if (!mc) throw std::runtime_error("Configuration error: open_clip_config.json has no model_cfg");
  OpenClipConfig c;
  if (!mc->get("embed_dim")) throw std::runtime_error("Configuration error: model_cfg.embed_dim missing");
  c.embed_dim = geti(mc, "embed_dim", 0);

  const json::Value* v = mc->get("vision_cfg");
  if (!v || !v->get("image_size")) throw std::runtime_error("Configuration error: vision_cfg.image_size missing");
  {
    const json::Value* x = v->get("attentional_pool");
    if (x && !x->is_null() && !(x->kind == json::Value::BOOL && !x->b))
      throw std::runtime_error("Configuration error: vision_cfg.attentional_pool is not supported yet");
  }
  TowerSpec& vs = c.vision;
  vs.tower = TOWER_VISION;
  vs.image_size = geti(v, "image_size", 224);
  const json::Value* timm = v->get("timm_model_name");
  if (timm && !timm->is_null()) {
    timm_siglip_spec(timm->as_str(""), v, vs);
    if (c.embed_dim != vs.width)
      throw std::runtime_error("Configuration error: timm_proj 'none' needs embed_dim == width");
    vs.embed_dim = c.embed_dim;
  } else {
    vs.patch_size = geti(v, "patch_size", 16);
    vs.width = geti(v, "width", 768);
    vs.layers = geti(v, "layers", 12);
    vs.heads = vs.width / geti(v, "head_width", 64);
    vs.mlp_width = (int)(vs.width * getd(v, "mlp_ratio", 4.0));
    vs.embed_dim = c.embed_dim;
    vs.act = act_from(*mc, v);
  }

  const json::Value* t = mc->get("text_cfg");
  if (!t || !t->get("context_length"))
    throw std::runtime_error("Configuration error: text_cfg.context_length missing");
  TowerSpec& ts = c.text;
  ts.tower = TOWER_TEXT;
  ts.context_length = geti(t, "context_length", 77);
  ts.vocab_size = geti(t, "vocab_size", 49408);
  ts.width = geti(t, "width", 512);
  ts.layers = geti(t, "layers", 12);
  ts.heads = geti(t, "heads", 8);
  ts.mlp_width = (int)(ts.width * getd(t, "mlp_ratio", 4.0));
  ts.embed_dim = c.embed_dim;
  ts.act = act_from(*mc, t);
  // The text engine builds open_clip's TextTransformer in its two exported forms: CLIP's (causal
  // mask, argmax / EOT pooling, projection matrix) and SigLIP2's (no_causal_mask, pool_type "last",
  // proj_bias, GELU tanh, norm eps 1e-6).  Other forms are refused, not mis-run.
  if (const json::Value* nk = t->get("norm_kwargs"))
    if (const json::Value* ep = nk->get("eps")) ts.ln_eps = (float)ep->as_num(1e-5);
  auto text_flag = [&](const char* key) {
    const json::Value* f = t->get(key);
    return f && !f->is_null() && f->as_bool(false);
  };
  auto text_str = [&](const char* key, const char* dflt) {
    const json::Value* f = t->get(key);
    return (f && !f->is_null()) ? f->as_str(dflt) : std::string(dflt);
  };
  ts.causal = !text_flag("no_causal_mask");
  ts.pool_last = text_str("pool_type", "argmax") == "last";
  ts.proj_bias = text_flag("proj_bias");
  const std::string pool = text_str("pool_type", "argmax");
  if (pool != "argmax" && pool != "last")
    ts.unsupported = "Configuration error: text_cfg.pool_type '" + pool +
                     "' is not supported (argmax / EOT or last-token pooling only)";
  else if (text_str("proj_type", "linear") != "linear")
    ts.unsupported = "Configuration error: text_cfg.proj_type '" + text_str("proj_type", "") + "' is not supported";
  else if (text_flag("embed_cls"))
    ts.unsupported = "Configuration error: text_cfg.embed_cls is not supported";
  else if (t->get("hf_model_name") && !t->get("hf_model_name")->is_null())
    ts.unsupported = "Configuration error: HF text towers (text_cfg.hf_model_name) are not supported";

  const json::Value* pc = root->get("preprocess_cfg");
  if (!pc) throw std::runtime_error("Configuration error: preprocess_cfg missing");
  const json::Value* mean = pc->get("mean");
  const json::Value* stdv = pc->get("std");
  if (!mean || !stdv || mean->arr.size() != 3 || stdv->arr.size() != 3)
    throw std::runtime_error("Configuration error: preprocess_cfg.mean/std must have 3 entries");
  for (int i = 0; i < 3; ++i) {
    c.pre.mean[i] = (float)mean->arr[i]->as_num(0);
    c.pre.stdv[i] = (float)stdv->arr[i]->as_num(1);
  }
  const json::Value* interp = pc->get("interpolation");
  if (interp && interp->kind == json::Value::STR) c.pre.interpolation = interp->str;
  const json::Value* rm = pc->get("resize_mode");
  if (rm && rm->kind == json::Value::STR) c.pre.resize_mode = rm->str;
  return c;
}

ModelConfig load_model_config(const std::string& path) {
  json::ValuePtr root = json::parse_file(path);
  ModelConfig m;
  if (const json::Value* v = root->get("tokenizer_needs_lowercase")) m.tokenizer_needs_lowercase = v->as_bool(false);
  if (const json::Value* v = root->get("activation_function"))
    if (v->kind == json::Value::STR) m.activation_function = v->str;
  if (const json::Value* v = root->get("logit_scale"))
    if (v->kind == json::Value::NUM) { m.has_logit_scale = true; m.logit_scale = (float)v->num; }
  if (const json::Value* v = root->get("logit_bias"))
    if (v->kind == json::Value::NUM) { m.has_logit_bias = true; m.logit_bias = (float)v->num; }
  if (const json::Value* v = root->get("pad_id"))
    if (v->kind == json::Value::NUM) m.pad_id = (long)v->num;
  return m;
}

}  // namespace clipgpu
