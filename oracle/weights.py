"""Deterministic counter-based weight generator (splitmix64) — TEST INFRASTRUCTURE.

No checkpoint can be fetched in this sandbox, so parity and benchmark runs use
weights regenerated from a seed.  The C++ engine mirrors this generator
bit-exactly (``clip-embedder-rs_amd/csrc/host/synth.cpp``); ``tests/`` check the
two against each other through ``clipgpu_synth_tensor``.

Element ``i`` of tensor ``name``::

    s   = mix64(seed ^ fnv1a64(name))
    z   = mix64(s + (i + 1) * 0x9E3779B97F4A7C15)          (mod 2**64)
    u   = f32(z >> 40) * 2**-23 - 1                          in [-1, 1), exact
    val = u * f32(amp) + f32(offset)                         two f32 roundings

``amp`` = std * sqrt(3) (uniform with the open_clip init std), computed in
double and rounded once to f32.  Init stds follow open_clip's
``VisionTransformer.init_parameters`` / ``TextTransformer.init_parameters``;
LayerNorm gains/biases and linear biases are perturbed away from 1/0 so that
every parameter is exercised by the parity tests.
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np

from .model_spec import VisionSpec, TextSpec

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & M64
    return h


def mix64_scalar(z: int) -> int:
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _mix64_np(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniform_pm1(seed: int, n: int) -> np.ndarray:
    """f32 values in [-1, 1) for counters 1..n of stream ``seed``."""
    s = np.uint64(seed & M64)
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = _mix64_np(s + idx * np.uint64(GOLDEN))
    u = (z >> np.uint64(40)).astype(np.float32)
    return u * np.float32(2.0 ** -23) - np.float32(1.0)


def synth_tensor(seed: int, name: str, shape, std: float, offset: float = 0.0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    ts = mix64_scalar((seed & M64) ^ fnv1a64(name))
    amp = np.float32(std * math.sqrt(3.0))
    v = uniform_pm1(ts, n) * amp + np.float32(offset)
    return v.astype(np.float32).reshape(shape)


# (name, shape, std, offset) — order is irrelevant (per-tensor streams).
ParamList = List[Tuple[str, Tuple[int, ...], float, float]]

LN_GAIN_STD = 0.1 / math.sqrt(3.0)   # gain uniform in 1 +- 0.1
LN_BIAS_STD = 0.05 / math.sqrt(3.0)  # bias uniform in +- 0.05
LIN_BIAS_STD = 0.02 / math.sqrt(3.0)


def _block_params(prefix: str, D: int, M: int, L: int) -> ParamList:
    attn_std = D ** -0.5
    proj_std = (D ** -0.5) * ((2 * L) ** -0.5)
    fc_std = (2 * D) ** -0.5
    return [
        (prefix + "ln_1.weight", (D,), LN_GAIN_STD, 1.0),
        (prefix + "ln_1.bias", (D,), LN_BIAS_STD, 0.0),
        (prefix + "attn.in_proj_weight", (3 * D, D), attn_std, 0.0),
        (prefix + "attn.in_proj_bias", (3 * D,), LIN_BIAS_STD, 0.0),
        (prefix + "attn.out_proj.weight", (D, D), proj_std, 0.0),
        (prefix + "attn.out_proj.bias", (D,), LIN_BIAS_STD, 0.0),
        (prefix + "ln_2.weight", (D,), LN_GAIN_STD, 1.0),
        (prefix + "ln_2.bias", (D,), LN_BIAS_STD, 0.0),
        (prefix + "mlp.c_fc.weight", (M, D), fc_std, 0.0),
        (prefix + "mlp.c_fc.bias", (M,), LIN_BIAS_STD, 0.0),
        (prefix + "mlp.c_proj.weight", (D, M), proj_std, 0.0),
        (prefix + "mlp.c_proj.bias", (D,), LIN_BIAS_STD, 0.0),
    ]


def _timm_block_params(prefix: str, D: int, M: int, L: int) -> ParamList:
    attn_std = D ** -0.5
    proj_std = (D ** -0.5) * ((2 * L) ** -0.5)
    fc_std = (2 * D) ** -0.5
    return [
        (prefix + "norm1.weight", (D,), LN_GAIN_STD, 1.0),
        (prefix + "norm1.bias", (D,), LN_BIAS_STD, 0.0),
        (prefix + "attn.qkv.weight", (3 * D, D), attn_std, 0.0),
        (prefix + "attn.qkv.bias", (3 * D,), LIN_BIAS_STD, 0.0),
        (prefix + "attn.proj.weight", (D, D), proj_std, 0.0),
        (prefix + "attn.proj.bias", (D,), LIN_BIAS_STD, 0.0),
        (prefix + "norm2.weight", (D,), LN_GAIN_STD, 1.0),
        (prefix + "norm2.bias", (D,), LN_BIAS_STD, 0.0),
        (prefix + "mlp.fc1.weight", (M, D), fc_std, 0.0),
        (prefix + "mlp.fc1.bias", (M,), LIN_BIAS_STD, 0.0),
        (prefix + "mlp.fc2.weight", (D, M), proj_std, 0.0),
        (prefix + "mlp.fc2.bias", (D,), LIN_BIAS_STD, 0.0),
    ]


def siglip_vision_param_list(v: VisionSpec) -> ParamList:
    """open_clip TimmModel (visual.trunk = timm VisionTransformer, global_pool 'map')."""
    D, p, M = v.width, v.patch_size, v.mlp_width
    t = "visual.trunk."
    out: ParamList = [
        (t + "patch_embed.proj.weight", (D, 3, p, p), (3 * p * p) ** -0.5, 0.0),
        (t + "patch_embed.proj.bias", (D,), LIN_BIAS_STD, 0.0),
        (t + "pos_embed", (1, v.grid * v.grid, D), D ** -0.5, 0.0),
    ]
    for i in range(v.layers):
        out += _timm_block_params(f"{t}blocks.{i}.", D, M, v.layers)
    a = t + "attn_pool."
    out += [
        (t + "norm.weight", (D,), LN_GAIN_STD, 1.0),
        (t + "norm.bias", (D,), LN_BIAS_STD, 0.0),
        (a + "latent", (1, 1, D), D ** -0.5, 0.0),
        (a + "q.weight", (D, D), D ** -0.5, 0.0),
        (a + "q.bias", (D,), LIN_BIAS_STD, 0.0),
        (a + "kv.weight", (2 * D, D), D ** -0.5, 0.0),
        (a + "kv.bias", (2 * D,), LIN_BIAS_STD, 0.0),
        (a + "proj.weight", (D, D), D ** -0.5, 0.0),
        (a + "proj.bias", (D,), LIN_BIAS_STD, 0.0),
        (a + "norm.weight", (D,), LN_GAIN_STD, 1.0),
        (a + "norm.bias", (D,), LN_BIAS_STD, 0.0),
        (a + "mlp.fc1.weight", (M, D), (2 * D) ** -0.5, 0.0),
        (a + "mlp.fc1.bias", (M,), LIN_BIAS_STD, 0.0),
        (a + "mlp.fc2.weight", (D, M), D ** -0.5, 0.0),
        (a + "mlp.fc2.bias", (D,), LIN_BIAS_STD, 0.0),
    ]
    return out


def vision_param_list(v: VisionSpec) -> ParamList:
    if v.family == "siglip":
        return siglip_vision_param_list(v)
    D, p = v.width, v.patch_size
    out: ParamList = [
        ("visual.conv1.weight", (D, 3, p, p), (3 * p * p) ** -0.5, 0.0),
        ("visual.class_embedding", (D,), D ** -0.5, 0.0),
        ("visual.positional_embedding", (v.tokens, D), D ** -0.5, 0.0),
        ("visual.ln_pre.weight", (D,), LN_GAIN_STD, 1.0),
        ("visual.ln_pre.bias", (D,), LN_BIAS_STD, 0.0),
    ]
    for i in range(v.layers):
        out += _block_params(f"visual.transformer.resblocks.{i}.", D, v.mlp_width, v.layers)
    out += [
        ("visual.ln_post.weight", (D,), LN_GAIN_STD, 1.0),
        ("visual.ln_post.bias", (D,), LN_BIAS_STD, 0.0),
        ("visual.proj", (D, v.embed_dim), D ** -0.5, 0.0),
    ]
    return out


def text_param_list(t: TextSpec) -> ParamList:
    D = t.width
    out: ParamList = [
        ("token_embedding.weight", (t.vocab_size, D), 0.02, 0.0),
        ("positional_embedding", (t.context_length, D), 0.01, 0.0),
    ]
    for i in range(t.layers):
        out += _block_params(f"transformer.resblocks.{i}.", D, t.mlp_width, t.layers)
    out += [
        ("ln_final.weight", (D,), LN_GAIN_STD, 1.0),
        ("ln_final.bias", (D,), LN_BIAS_STD, 0.0),
    ]
    if t.proj_bias:  # open_clip nn.Linear(width, embed_dim): weight [E, D] + bias
        out += [("text_projection.weight", (t.embed_dim, D), D ** -0.5, 0.0),
                ("text_projection.bias", (t.embed_dim,), 0.02, 0.0)]
    else:
        out += [("text_projection", (D, t.embed_dim), D ** -0.5, 0.0)]
    return out


def make_weights(params: ParamList, seed: int) -> Dict[str, np.ndarray]:
    return {n: synth_tensor(seed, n, s, std, off) for (n, s, std, off) in params}


def vision_weights(v: VisionSpec, seed: int) -> Dict[str, np.ndarray]:
    return make_weights(vision_param_list(v), seed)


def text_weights(t: TextSpec, seed: int) -> Dict[str, np.ndarray]:
    return make_weights(text_param_list(t), seed)


# Synthetic inputs shared by tests and bench -------------------------------

def synth_images_u8(seed: int, B: int, S: int) -> np.ndarray:
    """[B, S, S, 3] RGB u8 (HWC per image), uniform over 0..255."""
    ts = mix64_scalar((seed & M64) ^ fnv1a64("images_u8"))
    n = B * S * S * 3
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = _mix64_np(np.uint64(ts) + idx * np.uint64(GOLDEN))
    return (z >> np.uint64(56)).astype(np.uint8).reshape(B, S, S, 3)


def synth_token_ids(seed: int, B: int, T: int, vocab: int, bos: int, eot: int,
                    random_eot: bool = False) -> np.ndarray:
    """[B, T] int64: BOS, random ids in [0, vocab-3], EOT (at T-1 or random), pads 0."""
    ts = mix64_scalar((seed & M64) ^ fnv1a64("token_ids"))
    n = B * T
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = _mix64_np(np.uint64(ts) + idx * np.uint64(GOLDEN))
    ids = (z % np.uint64(vocab - 2)).astype(np.int64).reshape(B, T)
    ids[:, 0] = bos
    if random_eot:
        pos = 1 + (ids[:, 1] % (T - 1))
        for b in range(B):
            ids[b, pos[b]] = eot
            ids[b, pos[b] + 1:] = 0
    else:
        ids[:, T - 1] = eot
    return ids
