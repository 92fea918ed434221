// ONNX initializer reader: the reference's model folders hold the weights only
// inside visual.onnx / text.onnx (+ visual.onnx.data / text.onnx.data external
// data; src/model_manager.rs:8-18), exported by pull_onnx.py:170-195 from
// VisualWrapper / TextWrapper(model) -- so initializer names are the open_clip
// state-dict names behind a "model." prefix (model.visual.conv1.weight, ...).
//
// This is a minimal protobuf wire-format parser (no libprotobuf in the image):
// ModelProto.graph(7) -> GraphProto.initializer(5) TensorProto and nodes(1)
// (NodeProto input(1), output(2), name(3), op_type(4), attribute(5)).
// TensorProto: dims(1), data_type(2), float_data(4), int32_data(5), name(8),
// raw_data(9), double_data(10), external_data(13), data_location(14).
//
// Parameter resolution (checked against torch.onnx.export of an open_clip-
// structured model with the pull_onnx.py arguments, tests/onnx_export.py):
//   1. initializer named "<name>" or "model.<name>";
//   2. Identity-node aliases (the exporter de-duplicates identical tensors and
//      re-emits the parameter name as an Identity output);
//   3. constant-folded linear weights: an anonymous initializer ("onnx::MatMul_N",
//      stored pre-transposed [in][out]) consumed by the MatMul node of a module --
//      node "/visual/transformer/resblocks.3/mlp/c_fc/MatMul" -> "...mlp.c_fc.weight",
//      ".../attn/MatMul" -> "...attn.in_proj_weight"; Gemm with transB = 0 likewise;
//   4. folded token constants: open_clip's _expand_token(class_embedding).to(dtype)
//      becomes "onnx::Expand_N" [1,1,D] under the tower's Expand node, and
//      positional_embedding.to(dtype) becomes "onnx::Add_N" [T,D] under the tower
//      root's Add node (visual: "/visual/Add", text: "/Add"); for the timm trunk of
//      the SigLIP family: "/visual/trunk/Add" (pos_embed) and the attn_pool Expand
//      (latent).  timm Linear leaves (qkv, proj, fc1, fc2, q, kv) fold like c_fc.
// The graph is not otherwise interpreted: the engine implements the tower itself.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "model.hpp"

namespace clipgpu {

float half_to_float(uint16_t h);  // weights.cpp

namespace {

struct Mapped {
  const unsigned char* p = nullptr;
  size_t n = 0;
  explicit Mapped(const std::string& path) {
    int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("IO error: cannot open '" + path + "'");
    struct stat st;
    if (fstat(fd, &st) != 0) {
      ::close(fd);
      throw std::runtime_error("IO error: cannot stat '" + path + "'");
    }
    n = (size_t)st.st_size;
    if (n) {
      void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
      if (m == MAP_FAILED) {
        ::close(fd);
        throw std::runtime_error("IO error: mmap failed for '" + path + "'");
      }
      p = (const unsigned char*)m;
    }
    ::close(fd);
  }
  ~Mapped() {
    if (p) munmap((void*)p, n);
  }
  Mapped(const Mapped&) = delete;
  Mapped& operator=(const Mapped&) = delete;
};

struct Reader {
  const unsigned char* p;
  const unsigned char* e;
  bool done() const { return p >= e; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= e) throw std::runtime_error("Configuration error: truncated ONNX protobuf");
      const unsigned char b = *p++;
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    throw std::runtime_error("Configuration error: bad varint in ONNX protobuf");
  }
  Reader sub() {  // length-delimited payload
    const uint64_t n = varint();
    if (n > (uint64_t)(e - p)) throw std::runtime_error("Configuration error: truncated ONNX protobuf field");
    Reader r{p, p + n};
    p += n;
    return r;
  }
  void skip(int wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1: advance(8); break;
      case 2: sub(); break;
      case 5: advance(4); break;
      default: throw std::runtime_error("Configuration error: unsupported protobuf wire type");
    }
  }
  void advance(size_t n) {
    if (n > (size_t)(e - p)) throw std::runtime_error("Configuration error: truncated ONNX protobuf");
    p += n;
  }
};

enum OnnxType { OT_FLOAT = 1, OT_FLOAT16 = 10, OT_DOUBLE = 11, OT_BFLOAT16 = 16 };

struct TensorRec {
  std::string name;
  std::vector<int64_t> dims;
  int dtype = 0;
  const unsigned char* raw = nullptr;  // raw_data or the packed float/int32/double payload
  size_t raw_len = 0;
  int payload = 0;                     // 9 raw, 4 float_data, 5 int32_data, 10 double_data
  std::string ext_location;
  int64_t ext_offset = 0, ext_length = -1;
  bool external = false;
};

TensorRec parse_tensor(Reader r) {
  TensorRec t;
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int field = (int)(key >> 3), wt = (int)(key & 7);
    if (field == 1) {
      if (wt == 0) {
        t.dims.push_back((int64_t)r.varint());
      } else {
        Reader d = r.sub();
        while (!d.done()) t.dims.push_back((int64_t)d.varint());
      }
    } else if (field == 2 && wt == 0) {
      t.dtype = (int)r.varint();
    } else if (field == 8 && wt == 2) {
      Reader s = r.sub();
      t.name.assign((const char*)s.p, (size_t)(s.e - s.p));
    } else if ((field == 9 || field == 4 || field == 10) && wt == 2) {
      Reader s = r.sub();
      t.raw = s.p;
      t.raw_len = (size_t)(s.e - s.p);
      t.payload = field;
    } else if (field == 5 && wt == 2) {  // int32_data (packed): fp16/bf16 bits
      Reader s = r.sub();
      t.raw = s.p;
      t.raw_len = (size_t)(s.e - s.p);
      t.payload = 5;
    } else if (field == 13 && wt == 2) {  // StringStringEntryProto {key=1, value=2}
      Reader kv = r.sub();
      std::string k, v;
      while (!kv.done()) {
        const uint64_t kk = kv.varint();
        if ((kk >> 3) == 1 && (kk & 7) == 2) {
          Reader s = kv.sub();
          k.assign((const char*)s.p, (size_t)(s.e - s.p));
        } else if ((kk >> 3) == 2 && (kk & 7) == 2) {
          Reader s = kv.sub();
          v.assign((const char*)s.p, (size_t)(s.e - s.p));
        } else {
          kv.skip((int)(kk & 7));
        }
      }
      if (k == "location") t.ext_location = v;
      else if (k == "offset") t.ext_offset = std::stoll(v);
      else if (k == "length") t.ext_length = std::stoll(v);
    } else if (field == 14 && wt == 0) {
      t.external = r.varint() == 1;
    } else {
      r.skip(wt);
    }
  }
  if (!t.ext_location.empty()) t.external = true;
  return t;
}

struct NodeRec {
  std::string name, op;
  std::vector<std::string> inputs, outputs;
  int64_t transB = 0;
};

// Nodes; Constant nodes also yield a tensor named by their first output.
void parse_node(Reader r, std::vector<TensorRec>& tensors, std::vector<NodeRec>& nodes) {
  NodeRec n;
  std::vector<TensorRec> vals;
  while (!r.done()) {
    const uint64_t key = r.varint();
    const int field = (int)(key >> 3), wt = (int)(key & 7);
    auto str = [&](std::string& dst) {
      Reader s = r.sub();
      dst.assign((const char*)s.p, (size_t)(s.e - s.p));
    };
    if (field == 1 && wt == 2) {
      n.inputs.emplace_back();
      str(n.inputs.back());
    } else if (field == 2 && wt == 2) {
      n.outputs.emplace_back();
      str(n.outputs.back());
    } else if (field == 3 && wt == 2) {
      str(n.name);
    } else if (field == 4 && wt == 2) {
      str(n.op);
    } else if (field == 5 && wt == 2) {  // AttributeProto {name=1, i=3, t=5}
      Reader a = r.sub();
      std::string aname;
      int64_t ival = 0;
      TensorRec tr;
      bool has_t = false;
      while (!a.done()) {
        const uint64_t kk = a.varint();
        if ((kk >> 3) == 1 && (kk & 7) == 2) {
          Reader s = a.sub();
          aname.assign((const char*)s.p, (size_t)(s.e - s.p));
        } else if ((kk >> 3) == 3 && (kk & 7) == 0) {
          ival = (int64_t)a.varint();
        } else if ((kk >> 3) == 5 && (kk & 7) == 2) {
          tr = parse_tensor(a.sub());
          has_t = true;
        } else {
          a.skip((int)(kk & 7));
        }
      }
      if (has_t && aname == "value") vals.push_back(std::move(tr));
      if (aname == "transB") n.transB = ival;
    } else {
      r.skip(wt);
    }
  }
  if (n.op == "Constant" && !n.outputs.empty() && !vals.empty()) {
    vals[0].name = n.outputs[0];
    tensors.push_back(std::move(vals[0]));
  }
  nodes.push_back(std::move(n));
}

std::vector<TensorRec> parse_model(const unsigned char* p, size_t n, std::vector<NodeRec>& nodes) {
  std::vector<TensorRec> out;
  Reader m{p, p + n};
  bool graph_seen = false;
  while (!m.done()) {
    const uint64_t key = m.varint();
    const int field = (int)(key >> 3), wt = (int)(key & 7);
    if (field == 7 && wt == 2) {
      graph_seen = true;
      Reader g = m.sub();
      while (!g.done()) {
        const uint64_t gk = g.varint();
        const int gf = (int)(gk >> 3), gw = (int)(gk & 7);
        if (gf == 5 && gw == 2) out.push_back(parse_tensor(g.sub()));
        else if (gf == 1 && gw == 2) parse_node(g.sub(), out, nodes);
        else g.skip(gw);
      }
    } else {
      m.skip(wt);
    }
  }
  if (!graph_seen) throw std::runtime_error("Configuration error: no graph in ONNX model");
  return out;
}

std::string dir_of(const std::string& path) {
  const size_t s = path.find_last_of('/');
  return s == std::string::npos ? std::string(".") : path.substr(0, s);
}

// Decodes a tensor to f32 (row-major, ONNX dims order).
std::vector<float> decode(const TensorRec& t, const std::string& base_dir,
                          std::map<std::string, std::unique_ptr<Mapped>>& files) {
  int64_t n = 1;
  for (int64_t d : t.dims) n *= d;
  const unsigned char* src = t.raw;
  size_t len = t.raw_len;
  int payload = t.payload;
  if (t.external) {
    if (t.ext_location.empty() || t.ext_location.find("..") != std::string::npos || t.ext_location[0] == '/')
      throw std::runtime_error("Configuration error: bad external data location for '" + t.name + "'");
    auto& f = files[t.ext_location];
    if (!f) f.reset(new Mapped(base_dir + "/" + t.ext_location));
    const int64_t esz = t.dtype == OT_FLOAT ? 4 : t.dtype == OT_DOUBLE ? 8 : 2;
    const int64_t want = t.ext_length >= 0 ? t.ext_length : n * esz;
    if (t.ext_offset < 0 || (size_t)(t.ext_offset + want) > f->n)
      throw std::runtime_error("Configuration error: external data out of range for '" + t.name + "'");
    src = f->p + t.ext_offset;
    len = (size_t)want;
    payload = 9;
  }
  std::vector<float> out((size_t)n);
  auto need = [&](size_t bytes) {
    if (len != bytes) throw std::runtime_error("Configuration error: ONNX tensor '" + t.name + "' has " +
                                               std::to_string(len) + " data bytes, expected " + std::to_string(bytes));
  };
  if (t.dtype == OT_FLOAT && (payload == 9 || payload == 4)) {
    need((size_t)n * 4);
    std::memcpy(out.data(), src, (size_t)n * 4);
  } else if (t.dtype == OT_DOUBLE && (payload == 9 || payload == 10)) {
    need((size_t)n * 8);
    for (int64_t i = 0; i < n; ++i) {
      double d;
      std::memcpy(&d, src + 8 * i, 8);
      out[i] = (float)d;
    }
  } else if ((t.dtype == OT_FLOAT16 || t.dtype == OT_BFLOAT16) && payload == 9) {
    need((size_t)n * 2);
    for (int64_t i = 0; i < n; ++i) {
      uint16_t h;
      std::memcpy(&h, src + 2 * i, 2);
      if (t.dtype == OT_FLOAT16) {
        out[i] = half_to_float(h);
      } else {
        const uint32_t bits = (uint32_t)h << 16;
        std::memcpy(&out[i], &bits, 4);
      }
    }
  } else if ((t.dtype == OT_FLOAT16 || t.dtype == OT_BFLOAT16) && payload == 5) {  // varint int32_data
    Reader r{src, src + len};
    for (int64_t i = 0; i < n; ++i) {
      if (r.done()) throw std::runtime_error("Configuration error: short int32_data for '" + t.name + "'");
      const uint16_t h = (uint16_t)r.varint();
      if (t.dtype == OT_FLOAT16) {
        out[i] = half_to_float(h);
      } else {
        const uint32_t bits = (uint32_t)h << 16;
        std::memcpy(&out[i], &bits, 4);
      }
    }
  } else if (n == 0) {
  } else {
    throw std::runtime_error("Configuration error: unsupported ONNX tensor encoding for '" + t.name + "' (data_type " +
                             std::to_string(t.dtype) + ")");
  }
  return out;
}

// "/visual/transformer/resblocks.0/mlp/c_fc/MatMul" -> "visual.transformer.resblocks.0.mlp.c_fc"
std::string module_path(const std::string& node_name) {
  std::vector<std::string> parts;
  size_t i = 0;
  while (i <= node_name.size()) {
    const size_t j = node_name.find('/', i);
    const std::string part = node_name.substr(i, j == std::string::npos ? std::string::npos : j - i);
    if (!part.empty()) parts.push_back(part);
    if (j == std::string::npos) break;
    i = j + 1;
  }
  if (!parts.empty()) parts.pop_back();  // the op itself
  if (!parts.empty() && parts[0] == "model") parts.erase(parts.begin());
  std::string out;
  for (size_t k = 0; k < parts.size(); ++k) out += (k ? "." : "") + parts[k];
  return out;
}

}  // namespace

TensorMap load_onnx(const std::string& path, const TowerSpec& spec) {
  Mapped f(path);
  std::vector<NodeRec> nodes;
  std::vector<TensorRec> recs = parse_model(f.p, f.n, nodes);
  std::map<std::string, const TensorRec*> by_name;
  for (const TensorRec& t : recs) by_name.emplace(t.name, &t);
  // Identity aliases: output name -> tensor of its input (chains resolved in order)
  for (const NodeRec& n : nodes) {
    if (n.op != "Identity" || n.inputs.empty() || n.outputs.empty()) continue;
    auto it = by_name.find(n.inputs[0]);
    if (it != by_name.end()) by_name.emplace(n.outputs[0], it->second);
  }
  // constant-folded linear weights, keyed by parameter name; value = (tensor, stored [in][out])
  std::map<std::string, std::pair<const TensorRec*, bool>> folded;
  for (const NodeRec& n : nodes) {
    // folded class token / positional embedding (rule 4): first initializer input of the
    // tower root's Expand / Add node
    if ((n.op == "Expand" || n.op == "Add") && !n.inputs.empty()) {
      const std::string mod = module_path(n.name);
      std::string param;
      if (mod == "visual" || mod.empty())  // open_clip VisionTransformer / text root
        param = (mod.empty() ? std::string() : mod + ".") + (n.op == "Expand" ? "class_embedding" : "positional_embedding");
      else if (mod == "visual.trunk" && n.op == "Add")  // timm _pos_embed
        param = "visual.trunk.pos_embed";
      else if (mod.size() >= 9 && mod.compare(mod.size() - 9, 9, "attn_pool") == 0 && n.op == "Expand")
        param = mod + ".latent";  // timm AttentionPoolLatent latent.expand(B, -1, -1)
      if (!param.empty())
        for (const std::string& in : n.inputs) {
          auto it = by_name.find(in);
          if (it == by_name.end()) continue;
          folded.emplace(param, std::make_pair(it->second, false));
          break;
        }
      continue;
    }
    if ((n.op != "MatMul" && n.op != "Gemm") || n.inputs.size() < 2) continue;
    auto it = by_name.find(n.inputs[1]);
    if (it == by_name.end()) continue;
    const std::string mod = module_path(n.name);
    if (mod.empty()) continue;
    const size_t dot = mod.find_last_of('.');
    const std::string leaf = dot == std::string::npos ? mod : mod.substr(dot + 1);
    const bool tr = n.op == "MatMul" || n.transB == 0;
    // open_clip: attn (nn.MultiheadAttention in_proj), c_fc, c_proj, out_proj;
    // timm: attn.qkv, attn.proj, mlp.fc1, mlp.fc2, attn_pool.q / kv / proj
    static const char* linear_leaves[] = {"c_fc", "c_proj", "out_proj", "qkv", "proj", "fc1", "fc2", "q", "kv"};
    if (leaf == "attn") {
      folded.emplace(mod + ".in_proj_weight", std::make_pair(it->second, tr));
    } else {
      for (const char* lf : linear_leaves)
        if (leaf == lf) folded.emplace(mod + ".weight", std::make_pair(it->second, tr));
    }
  }
  auto find = [&](const std::string& name, bool& tr) -> const TensorRec* {
    tr = false;
    for (const std::string& cand : {"model." + name, name}) {
      auto it = by_name.find(cand);
      if (it != by_name.end()) return it->second;
    }
    auto fo = folded.find(name);
    if (fo != folded.end()) {
      tr = fo->second.second;
      return fo->second.first;
    }
    return nullptr;
  };
  const std::string base_dir = dir_of(path);
  std::map<std::string, std::unique_ptr<Mapped>> files;
  TensorMap out;
  for (const ParamDesc& p : tower_params(spec)) {
    bool tr = false;
    const TensorRec* t = find(p.name, tr);
    if (!t) {
      std::string some;
      int k = 0;
      for (auto& kv : by_name) {
        if (k++ == 6) break;
        some += (k > 1 ? ", " : "") + kv.first;
      }
      throw std::runtime_error("Configuration error: initializer '" + p.name + "' (or 'model." + p.name +
                               "') not found in " + path + " (" + std::to_string(by_name.size()) +
                               " tensors, e.g. " + some + ")");
    }
    std::vector<int64_t> want = p.shape;
    if (tr) {
      if (want.size() != 2) throw std::runtime_error("Shape error: folded weight '" + p.name + "' is not a matrix");
      std::swap(want[0], want[1]);
    }
    int64_t n = 1, wn = 1;
    for (int64_t d : t->dims) n *= d;
    for (int64_t d : want) wn *= d;
    // rank-1 parameters may come with squeezed / unit dims
    if (t->dims != want && !(p.shape.size() == 1 && n == wn))
      throw std::runtime_error("Shape error: ONNX tensor '" + t->name + "' for '" + p.name + "' has an unexpected shape");
    HostTensor h;
    h.shape = p.shape;
    std::vector<float> v = decode(*t, base_dir, files);
    if (tr) {
      const int64_t R = want[0], C = want[1];  // stored [R][C] = [in][out] -> [out][in]
      h.data.resize((size_t)(R * C));
      for (int64_t r = 0; r < R; ++r)
        for (int64_t c = 0; c < C; ++c) h.data[(size_t)(c * R + r)] = v[(size_t)(r * C + c)];
    } else {
      h.data = std::move(v);
    }
    out.emplace(p.name, std::move(h));
  }
  return out;
}

}  // namespace clipgpu
