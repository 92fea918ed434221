"""ONNX model folders for tests, made the way the reference makes them.

TEST INFRASTRUCTURE (not product).  pull_onnx.py:170-195 exports
VisualWrapper(model) / TextWrapper(model) -- model.encode_image / encode_text with
normalize=True -- via torch.onnx.export(input_names=["pixel_values"|"input_ids"],
output_names=[...], dynamic_axes={0: "batch_size"}, opset_version=18,
do_constant_folding=True).  open_clip itself cannot be installed here, so the
towers below restate open_clip's module tree with the SAME attribute names
(VisionTransformer: conv1, class_embedding, positional_embedding, ln_pre,
transformer.resblocks[i].{ln_1, attn (nn.MultiheadAttention), ln_2,
mlp.{c_fc, gelu, c_proj}}, ln_post, proj; CLIP text: token_embedding,
positional_embedding, transformer, ln_final, text_projection, attn_mask) and load
the seeded weights of oracle/weights.py, so the exported graphs carry the
initializer names, de-duplication and constant folding of a real export.

torch ships here without the `onnx` package, which the legacy (TorchScript)
exporter imports only to splice onnxscript custom functions into the proto;
these graphs have none, so that step is bypassed.  (The dynamo exporter needs
onnxscript, which is not installed.)
"""
import os
from collections import OrderedDict

import numpy as np
import torch
from torch import nn


class QuickGELU(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class ResidualAttentionBlock(nn.Module):
    def __init__(self, d, heads, mlp, act, eps=1e-5):
        super().__init__()
        self.ln_1 = nn.LayerNorm(d, eps=eps)
        self.attn = nn.MultiheadAttention(d, heads, batch_first=True)
        self.ln_2 = nn.LayerNorm(d, eps=eps)
        self.mlp = nn.Sequential(OrderedDict([("c_fc", nn.Linear(d, mlp)), ("gelu", act()),
                                              ("c_proj", nn.Linear(mlp, d))]))

    def forward(self, x, attn_mask=None):
        y = self.ln_1(x)
        x = x + self.attn(y, y, y, need_weights=False, attn_mask=attn_mask)[0]
        return x + self.mlp(self.ln_2(x))


class Transformer(nn.Module):
    def __init__(self, d, layers, heads, mlp, act, eps=1e-5):
        super().__init__()
        self.resblocks = nn.ModuleList([ResidualAttentionBlock(d, heads, mlp, act, eps) for _ in range(layers)])

    def forward(self, x, attn_mask=None):
        for r in self.resblocks:
            x = r(x, attn_mask=attn_mask)
        return x


def _act(name):
    return {"quick_gelu": QuickGELU, "gelu": nn.GELU, "gelu_tanh": lambda: nn.GELU(approximate="tanh")}[name]


class VisionTransformer(nn.Module):
    def __init__(self, v):
        super().__init__()
        D, P, G = v.width, v.patch_size, v.image_size // v.patch_size
        self.conv1 = nn.Conv2d(3, D, P, P, bias=False)
        self.class_embedding = nn.Parameter(torch.zeros(D))
        self.positional_embedding = nn.Parameter(torch.zeros(G * G + 1, D))
        self.ln_pre = nn.LayerNorm(D, eps=v.ln_eps)
        self.transformer = Transformer(D, v.layers, v.heads, v.mlp_width, _act(v.act))
        self.ln_post = nn.LayerNorm(D, eps=v.ln_eps)
        self.proj = nn.Parameter(torch.zeros(D, v.embed_dim))

    def forward(self, x):
        x = self.conv1(x).flatten(2).transpose(1, 2)
        cls = self.class_embedding.view(1, 1, -1).expand(x.shape[0], -1, -1).to(x.dtype)  # open_clip _expand_token
        x = torch.cat([cls, x], dim=1) + self.positional_embedding.to(x.dtype)
        x = self.transformer(self.ln_pre(x))
        return self.ln_post(x[:, 0]) @ self.proj


class ClipModel(nn.Module):
    def __init__(self, v, t):
        super().__init__()
        self.visual = VisionTransformer(v)
        self.token_embedding = nn.Embedding(t.vocab_size, t.width)
        self.positional_embedding = nn.Parameter(torch.zeros(t.context_length, t.width))
        self.transformer = Transformer(t.width, t.layers, t.heads, t.mlp_width, _act(t.act))
        self.ln_final = nn.LayerNorm(t.width, eps=t.ln_eps)
        self.text_projection = nn.Parameter(torch.zeros(t.width, t.embed_dim))
        mask = torch.full((t.context_length, t.context_length), float("-inf")).triu_(1)
        self.register_buffer("attn_mask", mask, persistent=False)

    def encode_image(self, x, normalize=False):
        f = self.visual(x)
        return nn.functional.normalize(f, dim=-1) if normalize else f

    def encode_text(self, ids, normalize=False):
        cast_dtype = torch.float32  # open_clip: self.transformer.get_cast_dtype()
        x = self.token_embedding(ids).to(cast_dtype)
        x = x + self.positional_embedding.to(cast_dtype)
        x = self.ln_final(self.transformer(x, attn_mask=self.attn_mask))
        x = x[torch.arange(x.shape[0]), ids.argmax(dim=-1)] @ self.text_projection
        return nn.functional.normalize(x, dim=-1) if normalize else x


# ---- timm SigLIP ViT trunk (open_clip TimmModel, timm_pool "map", timm_proj "none") ------------
# timm is not installed here: restated with timm's attribute names (VisionTransformer:
# patch_embed.proj, pos_embed, blocks[i].{norm1, attn.{qkv, proj}, norm2, mlp.{fc1, act, fc2}},
# norm, attn_pool.{latent, q, kv, proj, norm, mlp.{fc1, fc2}}) and forward order.

class TimmMlp(nn.Module):
    def __init__(self, d, hidden):
        super().__init__()
        self.fc1 = nn.Linear(d, hidden)
        self.act = nn.GELU(approximate="tanh")
        self.fc2 = nn.Linear(hidden, d)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class TimmAttention(nn.Module):
    def __init__(self, d, heads):
        super().__init__()
        self.heads = heads
        self.qkv = nn.Linear(d, 3 * d)
        self.proj = nn.Linear(d, d)

    def forward(self, x):
        B, N, C = x.shape
        qkv = self.qkv(x).reshape(B, N, 3, self.heads, C // self.heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv.unbind(0)
        x = nn.functional.scaled_dot_product_attention(q, k, v)
        return self.proj(x.transpose(1, 2).reshape(B, N, C))


class TimmBlock(nn.Module):
    def __init__(self, d, heads, hidden):
        super().__init__()
        self.norm1 = nn.LayerNorm(d, eps=1e-6)
        self.attn = TimmAttention(d, heads)
        self.norm2 = nn.LayerNorm(d, eps=1e-6)
        self.mlp = TimmMlp(d, hidden)

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        return x + self.mlp(self.norm2(x))


class PatchEmbed(nn.Module):
    def __init__(self, p, d):
        super().__init__()
        self.proj = nn.Conv2d(3, d, p, p, bias=True)

    def forward(self, x):
        return self.proj(x).flatten(2).transpose(1, 2)


class AttentionPoolLatent(nn.Module):
    def __init__(self, d, heads, hidden):
        super().__init__()
        self.heads = heads
        self.latent = nn.Parameter(torch.zeros(1, 1, d))
        self.q = nn.Linear(d, d)
        self.kv = nn.Linear(d, 2 * d)
        self.proj = nn.Linear(d, d)
        self.norm = nn.LayerNorm(d, eps=1e-6)
        self.mlp = TimmMlp(d, hidden)

    def forward(self, x):
        B, N, C = x.shape
        hd = C // self.heads
        q = self.q(self.latent.expand(B, -1, -1)).reshape(B, 1, self.heads, hd).transpose(1, 2)
        kv = self.kv(x).reshape(B, N, 2, self.heads, hd).permute(2, 0, 3, 1, 4)
        k, v = kv.unbind(0)
        x = nn.functional.scaled_dot_product_attention(q, k, v)
        x = self.proj(x.transpose(1, 2).reshape(B, 1, C))
        x = x + self.mlp(self.norm(x))
        return x[:, 0]


class TimmSiglipViT(nn.Module):
    def __init__(self, v):
        super().__init__()
        D = v.width
        self.patch_embed = PatchEmbed(v.patch_size, D)
        self.pos_embed = nn.Parameter(torch.zeros(1, v.grid * v.grid, D))
        self.blocks = nn.ModuleList([TimmBlock(D, v.heads, v.mlp_width) for _ in range(v.layers)])
        self.norm = nn.LayerNorm(D, eps=1e-6)
        self.attn_pool = AttentionPoolLatent(D, v.heads, v.mlp_width)

    def forward(self, x):
        x = self.patch_embed(x)
        x = x + self.pos_embed
        for b in self.blocks:
            x = b(x)
        return self.attn_pool(self.norm(x))


class TimmModel(nn.Module):  # open_clip TimmModel with an empty head (timm_proj "none")
    def __init__(self, v):
        super().__init__()
        self.trunk = TimmSiglipViT(v)

    def forward(self, x):
        return self.trunk(x)


class SiglipVisionOnly(nn.Module):
    def __init__(self, v):
        super().__init__()
        self.visual = TimmModel(v)

    def encode_image(self, x, normalize=False):
        f = self.visual(x)
        return nn.functional.normalize(f, dim=-1) if normalize else f


def build_siglip_vision(v, seed):
    from oracle import weights
    m = SiglipVisionOnly(v).eval()
    P = weights.vision_weights(v, seed)
    sd = m.state_dict()
    assert set(sd) == set(P), set(sd) ^ set(P)
    m.load_state_dict({k: torch.from_numpy(np.asarray(P[k], np.float32)) for k in sd})
    return m


def export_siglip_visual(d, v, seed, external=False):
    import warnings
    m = build_siglip_vision(v, seed)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _export(VisualWrapper(m), torch.randn(2, 3, v.image_size, v.image_size), os.path.join(d, "visual.onnx"),
                "pixel_values", "image_embeddings")
    if external:
        externalize(os.path.join(d, "visual.onnx"))
    return m


class SiglipTextOnly(nn.Module):
    """open_clip TextTransformer in its SigLIP2 form (text_cfg no_causal_mask, pool_type "last",
    proj_bias, GELU tanh, norm eps 1e-6): no attention mask, x[:, -1] after ln_final, nn.Linear
    projection."""

    def __init__(self, t):
        super().__init__()
        self.token_embedding = nn.Embedding(t.vocab_size, t.width)
        self.positional_embedding = nn.Parameter(torch.zeros(t.context_length, t.width))
        self.transformer = Transformer(t.width, t.layers, t.heads, t.mlp_width, _act(t.act), t.ln_eps)
        self.ln_final = nn.LayerNorm(t.width, eps=t.ln_eps)
        self.text_projection = nn.Linear(t.width, t.embed_dim)

    def encode_text(self, ids, normalize=False):
        x = self.token_embedding(ids) + self.positional_embedding
        x = self.ln_final(self.transformer(x))
        x = self.text_projection(x[:, -1])
        return nn.functional.normalize(x, dim=-1) if normalize else x


def build_siglip_text(t, seed):
    from oracle import weights
    m = SiglipTextOnly(t).eval()
    P = weights.text_weights(t, seed)
    sd = m.state_dict()
    assert set(sd) == set(P), set(sd) ^ set(P)
    m.load_state_dict({k: torch.from_numpy(np.asarray(P[k], np.float32)) for k in sd})
    return m


def export_siglip_text(d, t, seed, external=False):
    import warnings
    m = build_siglip_text(t, seed)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _export(TextWrapper(m), torch.randint(0, t.vocab_size, (2, t.context_length)), os.path.join(d, "text.onnx"),
                "input_ids", "text_embeddings")
    if external:
        externalize(os.path.join(d, "text.onnx"))
    return m


class VisualWrapper(nn.Module):  # pull_onnx.py VisualWrapper
    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, x):
        return self.model.encode_image(x, normalize=True)


class TextWrapper(nn.Module):  # pull_onnx.py TextWrapper
    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, x):
        return self.model.encode_text(x, normalize=True)


def build_model(v, t, seed):
    """ClipModel with oracle/weights.py's seeded parameters (open_clip names)."""
    from oracle import weights
    m = ClipModel(v, t).eval()
    P = dict(weights.vision_weights(v, seed))
    P.update(weights.text_weights(t, seed))
    sd = m.state_dict()
    missing = set(sd) - set(P)
    assert not missing, missing
    m.load_state_dict({k: torch.from_numpy(np.asarray(P[k], np.float32)) for k in sd})
    return m


def _export(module, dummy, path, in_name, out_name):
    from torch.onnx._internal.torchscript_exporter import onnx_proto_utils, utils
    saved = onnx_proto_utils._add_onnxscript_fn
    onnx_proto_utils._add_onnxscript_fn = lambda model_bytes, custom_opsets: model_bytes
    saved_u = getattr(utils, "_add_onnxscript_fn", None)
    if saved_u is not None:
        utils._add_onnxscript_fn = onnx_proto_utils._add_onnxscript_fn
    try:
        torch.onnx.export(module, dummy, path, input_names=[in_name], output_names=[out_name],
                          dynamic_axes={in_name: {0: "batch_size"}, out_name: {0: "batch_size"}},
                          opset_version=18, do_constant_folding=True, dynamo=False)
    finally:
        onnx_proto_utils._add_onnxscript_fn = saved
        if saved_u is not None:
            utils._add_onnxscript_fn = saved_u


def export_model_dir(d, v, t, seed, external=False):
    """Writes visual.onnx / text.onnx into d (plus .onnx.data when external)."""
    import warnings
    m = build_model(v, t, seed)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _export(VisualWrapper(m), torch.randn(2, 3, v.image_size, v.image_size), os.path.join(d, "visual.onnx"),
                "pixel_values", "image_embeddings")
        _export(TextWrapper(m), torch.randint(0, t.vocab_size, (2, t.context_length)), os.path.join(d, "text.onnx"),
                "input_ids", "text_embeddings")
    if external:
        for name in ("visual.onnx", "text.onnx"):
            externalize(os.path.join(d, name))
    return m


# ---- minimal protobuf wire format (field rewrites only) ------------------------------------

def _varint(b, i):
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, i


def _enc_varint(v):
    out = bytearray()
    while True:
        c = v & 0x7F
        v >>= 7
        if v:
            out.append(c | 0x80)
        else:
            out.append(c)
            return bytes(out)


def _fields(b):
    """(field, wire_type, value, raw_span_bytes) for each top-level field."""
    i = 0
    while i < len(b):
        start = i
        k, i = _varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 2:
            n, i = _varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        else:
            raise ValueError("wire type")
        yield f, wt, v, b[start:i]


def _len_field(f, payload):
    return _enc_varint((f << 3) | 2) + _enc_varint(len(payload)) + payload


def externalize(path):
    """Moves every initializer's raw_data into <path>.data (external_data entries, data_location=1),
    as torch does for > 2 GB exports and as the reference's model folders ship them."""
    data_name = os.path.basename(path) + ".data"
    blob = bytearray()
    model = open(path, "rb").read()
    out_model = bytearray()
    for f, wt, v, raw in _fields(model):
        if f != 7:
            out_model += raw
            continue
        graph = bytearray()
        for gf, gw, gv, graw in _fields(v):
            if gf != 5:
                graph += graw
                continue
            tensor = bytearray()
            data = None
            for tf, tw, tv, traw in _fields(gv):
                if tf == 9:
                    data = bytes(tv)
                else:
                    tensor += traw
            if data is not None:
                off = len(blob)
                blob += data
                while len(blob) % 64:
                    blob += b"\0"
                for key, val in (("location", data_name), ("offset", str(off)), ("length", str(len(data)))):
                    entry = _len_field(1, key.encode()) + _len_field(2, val.encode())
                    tensor += _len_field(13, entry)
                tensor += _enc_varint((14 << 3) | 0) + _enc_varint(1)
            graph += _len_field(5, bytes(tensor))
        out_model += _len_field(7, bytes(graph))
    with open(path, "wb") as fh:
        fh.write(bytes(out_model))
    with open(os.path.join(os.path.dirname(path), data_name), "wb") as fh:
        fh.write(bytes(blob))


def initializer_names(path):
    names = []
    for f, wt, v, raw in _fields(open(path, "rb").read()):
        if f == 7:
            for gf, gw, gv, graw in _fields(v):
                if gf == 5:
                    for tf, tw, tv, traw in _fields(gv):
                        if tf == 8:
                            names.append(bytes(tv).decode())
    return names
