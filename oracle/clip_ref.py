"""numpy restatement of the reference's ONNX graphs — TEST INFRASTRUCTURE.

``pull_onnx.py:53-59`` exports ``VisualWrapper.forward = model.encode_image(x,
normalize=True)`` and ``pull_onnx.py:62-68`` exports ``TextWrapper.forward =
model.encode_text(x, normalize=True)`` (open-clip-torch 3.2.0, ``pull_onnx.py:7``);
the crate runs them verbatim (``src/vision.rs:108-113``, ``src/text.rs:156-166``)
and returns the graph output as the embedding (``README.md:81-82``: "already l2
normalized").  This module restates that arithmetic in float64 (default) or
float32 numpy.  Pinned against HF ``transformers`` CLIP / Siglip (tests/test_cpu_oracle.py).
"""
from __future__ import annotations

from typing import Dict

import numpy as np

from .model_spec import VisionSpec, TextSpec


def layer_norm(x, w, b, eps):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * w + b


def act_fn(name: str, x):
    if name == "quick_gelu":          # open_clip QuickGELU: x * sigmoid(1.702 x)
        return x / (1.0 + np.exp(-1.702 * x))
    if name == "gelu":                # nn.GELU() exact erf form
        from scipy.special import erf
        return 0.5 * x * (1.0 + erf(x / np.sqrt(2.0)))
    if name == "gelu_tanh":
        return 0.5 * x * (1.0 + np.tanh(np.sqrt(2.0 / np.pi) * (x + 0.044715 * x ** 3)))
    raise ValueError(name)


def softmax(x, axis=-1):
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True)


def l2_normalize(x, eps=1e-12):
    """torch.nn.functional.normalize(x, dim=-1): x / max(||x||_2, eps)."""
    n = np.sqrt((x * x).sum(-1, keepdims=True))
    return x / np.maximum(n, eps)


def _resblock(P, pre, x, heads, act, eps, causal):
    B, N, D = x.shape
    d = D // heads
    h = layer_norm(x, P[pre + "ln_1.weight"], P[pre + "ln_1.bias"], eps)
    qkv = h @ P[pre + "attn.in_proj_weight"].T + P[pre + "attn.in_proj_bias"]
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
    q = q.reshape(B, N, heads, d).transpose(0, 2, 1, 3)
    k = k.reshape(B, N, heads, d).transpose(0, 2, 1, 3)
    v = v.reshape(B, N, heads, d).transpose(0, 2, 1, 3)
    s = (q @ k.transpose(0, 1, 3, 2)) * (1.0 / np.sqrt(d))
    if causal:
        mask = np.triu(np.ones((N, N), dtype=bool), 1)
        s = np.where(mask, -np.inf, s)
    o = softmax(s) @ v
    o = o.transpose(0, 2, 1, 3).reshape(B, N, D)
    x = x + o @ P[pre + "attn.out_proj.weight"].T + P[pre + "attn.out_proj.bias"]
    h = layer_norm(x, P[pre + "ln_2.weight"], P[pre + "ln_2.bias"], eps)
    h = act_fn(act, h @ P[pre + "mlp.c_fc.weight"].T + P[pre + "mlp.c_fc.bias"])
    x = x + h @ P[pre + "mlp.c_proj.weight"].T + P[pre + "mlp.c_proj.bias"]
    return x


def _cast(P: Dict[str, np.ndarray], dtype):
    return {k: np.asarray(v, dtype=dtype) for k, v in P.items()}


def _timm_block(P, pre, x, heads, act, eps):
    """timm Block (norm1 -> Attention(qkv, proj) -> +, norm2 -> Mlp(fc1, act, fc2) -> +) written as
    the open_clip block with the fused qkv as in_proj: identical arithmetic."""
    Q = {pre + "ln_1.weight": P[pre + "norm1.weight"], pre + "ln_1.bias": P[pre + "norm1.bias"],
         pre + "attn.in_proj_weight": P[pre + "attn.qkv.weight"], pre + "attn.in_proj_bias": P[pre + "attn.qkv.bias"],
         pre + "attn.out_proj.weight": P[pre + "attn.proj.weight"], pre + "attn.out_proj.bias": P[pre + "attn.proj.bias"],
         pre + "ln_2.weight": P[pre + "norm2.weight"], pre + "ln_2.bias": P[pre + "norm2.bias"],
         pre + "mlp.c_fc.weight": P[pre + "mlp.fc1.weight"], pre + "mlp.c_fc.bias": P[pre + "mlp.fc1.bias"],
         pre + "mlp.c_proj.weight": P[pre + "mlp.fc2.weight"], pre + "mlp.c_proj.bias": P[pre + "mlp.fc2.bias"]}
    return _resblock(Q, pre, x, heads, act, eps, False)


def encode_image_siglip(P: Dict[str, np.ndarray], v: VisionSpec, pixels: np.ndarray,
                        dtype=np.float64, normalize: bool = True) -> np.ndarray:
    """open_clip TimmModel over a timm SigLIP ViT (global_pool 'map', timm_proj 'none') + normalize.
    timm VisionTransformer: patch_embed (conv, bias) -> + pos_embed (no class token, no norm_pre)
    -> blocks -> norm -> AttentionPoolLatent: q = latent Wq, [k|v] = x Wkv, per-head softmax
    attention, proj, x + mlp(norm(x)), token 0."""
    P = _cast(P, dtype)
    x = np.asarray(pixels, dtype=dtype)
    B = x.shape[0]
    p, g, D, H = v.patch_size, v.grid, v.width, v.heads
    d = D // H
    t, a = "visual.trunk.", "visual.trunk.attn_pool."
    patches = x.reshape(B, 3, g, p, g, p).transpose(0, 2, 4, 1, 3, 5).reshape(B, g * g, 3 * p * p)
    x = patches @ P[t + "patch_embed.proj.weight"].reshape(D, 3 * p * p).T + P[t + "patch_embed.proj.bias"]
    x = x + P[t + "pos_embed"][0]
    for i in range(v.layers):
        x = _timm_block(P, f"{t}blocks.{i}.", x, H, v.act, v.ln_eps)
    x = layer_norm(x, P[t + "norm.weight"], P[t + "norm.bias"], v.ln_eps)
    q = (P[a + "latent"].reshape(1, D) @ P[a + "q.weight"].T + P[a + "q.bias"]).reshape(H, d)
    kv = x @ P[a + "kv.weight"].T + P[a + "kv.bias"]                       # [B, N, 2D]
    k = kv[..., :D].reshape(B, -1, H, d)
    vv = kv[..., D:].reshape(B, -1, H, d)
    s = np.einsum("hd,bnhd->bhn", q, k) / np.sqrt(d)
    o = np.einsum("bhn,bnhd->bhd", softmax(s), vv).reshape(B, D)
    y = o @ P[a + "proj.weight"].T + P[a + "proj.bias"]
    h = act_fn(v.act, layer_norm(y, P[a + "norm.weight"], P[a + "norm.bias"], v.ln_eps) @ P[a + "mlp.fc1.weight"].T
               + P[a + "mlp.fc1.bias"])
    y = y + h @ P[a + "mlp.fc2.weight"].T + P[a + "mlp.fc2.bias"]
    return l2_normalize(y) if normalize else y


def encode_image(P: Dict[str, np.ndarray], v: VisionSpec, pixels: np.ndarray,
                 dtype=np.float64, normalize: bool = True) -> np.ndarray:
    """open_clip VisionTransformer.forward + normalize.  pixels: [B,3,S,S] normalised f32."""
    if v.family == "siglip":
        return encode_image_siglip(P, v, pixels, dtype, normalize)
    P = _cast(P, dtype)
    x = np.asarray(pixels, dtype=dtype)
    B = x.shape[0]
    p, g, D = v.patch_size, v.grid, v.width
    # conv1 (kernel = stride = p, no bias) == per-patch matmul
    patches = x.reshape(B, 3, g, p, g, p).transpose(0, 2, 4, 1, 3, 5).reshape(B, g * g, 3 * p * p)
    x = patches @ P["visual.conv1.weight"].reshape(D, 3 * p * p).T
    cls = np.broadcast_to(P["visual.class_embedding"], (B, 1, D))
    x = np.concatenate([cls, x], axis=1) + P["visual.positional_embedding"]
    x = layer_norm(x, P["visual.ln_pre.weight"], P["visual.ln_pre.bias"], v.ln_eps)
    for i in range(v.layers):
        x = _resblock(P, f"visual.transformer.resblocks.{i}.", x, v.heads, v.act, v.ln_eps, False)
    x = layer_norm(x, P["visual.ln_post.weight"], P["visual.ln_post.bias"], v.ln_eps)
    pooled = x[:, 0]                                  # pool_type 'tok' (CLS)
    out = pooled @ P["visual.proj"]
    return l2_normalize(out) if normalize else out


def encode_text(P: Dict[str, np.ndarray], t: TextSpec, ids: np.ndarray,
                dtype=np.float64, normalize: bool = True) -> np.ndarray:
    """open_clip TextTransformer.forward (transformer.py: token + positional embedding, the
    resblocks with the causal mask unless no_causal_mask, ln_final, text_global_pool, projection)
    + normalize.  CLIP: causal, argmax / EOT pooling, projection matrix.  SigLIP2: no mask,
    pool_type "last" (x[:, -1], the final context position, padding included), nn.Linear
    projection with bias.  ids: [B,T] int64."""
    P = _cast(P, dtype)
    ids = np.asarray(ids, dtype=np.int64)
    B, T = ids.shape
    x = P["token_embedding.weight"][ids] + P["positional_embedding"][:T]
    for i in range(t.layers):
        x = _resblock(P, f"transformer.resblocks.{i}.", x, t.heads, t.act, t.ln_eps, t.causal)
    x = layer_norm(x, P["ln_final.weight"], P["ln_final.bias"], t.ln_eps)
    if t.pool == "last":
        pooled = x[:, -1]
    else:
        pooled = x[np.arange(B), ids.argmax(-1)]      # first occurrence of the max id (EOT)
    if t.proj_bias:
        out = pooled @ P["text_projection.weight"].T + P["text_projection.bias"]
    else:
        out = pooled @ P["text_projection"]
    return l2_normalize(out) if normalize else out


def cosine_rows(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return (a * b).sum(-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))
