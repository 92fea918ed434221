"""Architecture spec derived from a model dir's ``open_clip_config.json``.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``).

The reference parses only ``embed_dim``, ``vision_cfg.{image_size,layers?,width?}``
and ``text_cfg.{context_length,hf_tokenizer_name?}`` (``src/config.rs:29-47``)
because everything else is baked into the ONNX graphs.  The graphs themselves are
open_clip ``VisionTransformer`` / ``TextTransformer`` modules exported by
``pull_onnx.py:53-68``; their defaults (head_width 64, mlp_ratio 4, LayerNorm eps
1e-5, CLS-token pooling, argmax/EOT text pooling, QuickGELU iff
``model_cfg.quick_gelu``) are restated here.  The C++ engine parses the same file
independently (``csrc/host/config.cpp``).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, asdict


@dataclass(frozen=True)
class VisionSpec:
    image_size: int
    patch_size: int
    width: int
    layers: int
    heads: int
    mlp_width: int
    embed_dim: int
    act: str            # "quick_gelu" | "gelu" | "gelu_tanh"
    ln_eps: float = 1e-5
    # "clip": open_clip VisionTransformer (CLS token, ln_pre, CLS pooling, proj);
    # "siglip": timm ViT trunk of open_clip TimmModel (no CLS, no pre-norm, patch-conv bias,
    # final norm, MAP attention-pool head, timm_proj "none")
    family: str = "clip"

    @property
    def grid(self) -> int:
        return self.image_size // self.patch_size

    @property
    def tokens(self) -> int:
        return self.grid * self.grid + (1 if self.family == "clip" else 0)  # + CLS

    @property
    def head_dim(self) -> int:
        return self.width // self.heads


@dataclass(frozen=True)
class TextSpec:
    context_length: int
    vocab_size: int
    width: int
    layers: int
    heads: int
    mlp_width: int
    embed_dim: int
    act: str
    ln_eps: float = 1e-5
    # open_clip TextTransformer forms: CLIP's (causal mask, argmax / EOT pooling, projection
    # matrix without bias) and SigLIP2's (no_causal_mask, pool_type "last": the final context
    # position, padding included; text_projection an nn.Linear with bias)
    causal: bool = True
    pool: str = "argmax"        # "argmax" | "last"
    proj_bias: bool = False

    @property
    def head_dim(self) -> int:
        return self.width // self.heads


def _act(model_cfg: dict, sub: dict) -> str:
    if sub.get("act_layer") in ("gelu_tanh", "gelu_pytorch_tanh"):
        return "gelu_tanh"
    if (sub.get("act_kwargs") or {}).get("approximate") == "tanh":  # open_clip nn.GELU(approximate="tanh")
        return "gelu_tanh"
    return "quick_gelu" if model_cfg.get("quick_gelu", False) else "gelu"


# timm SigLIP ViTs as open_clip TimmModel builds them (timm_model_name -> patch, width, depth,
# heads, mlp hidden): global_pool "map", GELU(tanh), LayerNorm eps 1e-6, no class token,
# no pre-norm, patch-embedding conv with bias.
TIMM_SIGLIP = {}
for _res in (224, 256, 384, 512):
    TIMM_SIGLIP[f"vit_base_patch16_siglip_{_res}"] = (16, 768, 12, 12, 3072)
for _res in (256, 384):
    TIMM_SIGLIP[f"vit_large_patch16_siglip_{_res}"] = (16, 1024, 24, 16, 4096)
    TIMM_SIGLIP[f"vit_giantopt_patch16_siglip_{_res}"] = (16, 1536, 40, 16, 6144)
for _res in (224, 378, 384):
    TIMM_SIGLIP[f"vit_so400m_patch14_siglip_{_res}"] = (14, 1152, 27, 16, 4304)
for _res in (256, 384, 512):
    TIMM_SIGLIP[f"vit_so400m_patch16_siglip_{_res}"] = (16, 1152, 27, 16, 4304)


def _siglip_vision_spec(model_cfg: dict, v: dict) -> VisionSpec:
    name = v["timm_model_name"]
    if name not in TIMM_SIGLIP:
        raise ValueError(f"timm model {name} is not supported")
    if v.get("timm_pool", "map") != "map" or v.get("timm_proj", "none") not in ("none", None):
        raise ValueError("only timm_pool 'map' with timm_proj 'none' is supported")
    patch, width, layers, heads, mlp = TIMM_SIGLIP[name]
    dims = v.get("clipgpu_dims", {})  # synthetic test configs only: explicit (reduced) dims
    patch, width = int(dims.get("patch_size", patch)), int(dims.get("width", width))
    layers, heads, mlp = int(dims.get("layers", layers)), int(dims.get("heads", heads)), int(dims.get("mlp_width", mlp))
    if int(model_cfg["embed_dim"]) != width:
        raise ValueError("timm_proj 'none' needs embed_dim == width")
    return VisionSpec(image_size=int(v["image_size"]), patch_size=patch, width=width, layers=layers, heads=heads,
                      mlp_width=mlp, embed_dim=width, act="gelu_tanh", ln_eps=1e-6, family="siglip")


def vision_spec_from_cfg(model_cfg: dict) -> VisionSpec:
    v = model_cfg["vision_cfg"]
    if v.get("timm_model_name"):
        return _siglip_vision_spec(model_cfg, v)
    for unsupported in ("attentional_pool", "attn_pooler_queries"):
        if v.get(unsupported):
            raise ValueError(f"vision_cfg.{unsupported} is not supported by this oracle")
    width = int(v.get("width", 768))
    head_width = int(v.get("head_width", 64))
    return VisionSpec(
        image_size=int(v["image_size"]),
        patch_size=int(v.get("patch_size", 16)),
        width=width,
        layers=int(v.get("layers", 12)),
        heads=width // head_width,
        mlp_width=int(width * float(v.get("mlp_ratio", 4.0))),
        embed_dim=int(model_cfg["embed_dim"]),
        act=_act(model_cfg, v),
    )


def text_spec_from_cfg(model_cfg: dict) -> TextSpec:
    t = model_cfg["text_cfg"]
    if t.get("hf_model_name"):
        raise ValueError("text_cfg.hf_model_name (HF text towers) is not supported by this oracle")
    pool = t.get("pool_type", "argmax")
    if pool not in ("argmax", "last"):
        raise ValueError(f"text_cfg.pool_type {pool!r} is not supported by this oracle")
    if t.get("proj_type", "linear") != "linear" or t.get("embed_cls"):
        raise ValueError("only a linear text projection without a CLS embedding is supported by this oracle")
    width = int(t.get("width", 512))
    return TextSpec(
        context_length=int(t.get("context_length", 77)),
        vocab_size=int(t.get("vocab_size", 49408)),
        width=width,
        layers=int(t.get("layers", 12)),
        heads=int(t.get("heads", 8)),
        mlp_width=int(width * float(t.get("mlp_ratio", 4.0))),
        embed_dim=int(model_cfg["embed_dim"]),
        act=_act(model_cfg, t),
        ln_eps=float((t.get("norm_kwargs") or {}).get("eps", 1e-5)),
        causal=not t.get("no_causal_mask", False),
        pool=pool,
        proj_bias=bool(t.get("proj_bias", False)),
    )


def load_model_dir(model_dir: str):
    with open(os.path.join(model_dir, "open_clip_config.json")) as f:
        oc = json.load(f)
    mc = oc["model_cfg"]
    return vision_spec_from_cfg(mc), text_spec_from_cfg(mc), oc


# ---------------------------------------------------------------------------
# Canonical configs used by tests and bench (open_clip_config.json contents).
# ---------------------------------------------------------------------------

OPENAI_MEAN = [0.48145466, 0.4578275, 0.40821073]
OPENAI_STD = [0.26862954, 0.26130258, 0.27577711]

VIT_B_32_CFG = {
    "model_cfg": {
        "embed_dim": 512,
        "quick_gelu": True,
        "vision_cfg": {"image_size": 224, "layers": 12, "width": 768, "patch_size": 32},
        "text_cfg": {"context_length": 77, "vocab_size": 49408, "width": 512,
                     "heads": 8, "layers": 12},
    },
    "preprocess_cfg": {"mean": OPENAI_MEAN, "std": OPENAI_STD},
}

# Small config with the same structure, for fast oracle/GPU parity cases.
TINY_CFG = {
    "model_cfg": {
        "embed_dim": 64,
        "quick_gelu": True,
        "vision_cfg": {"image_size": 64, "layers": 2, "width": 128, "patch_size": 16},
        "text_cfg": {"context_length": 16, "vocab_size": 1000, "width": 128,
                     "heads": 2, "layers": 2},
    },
    "preprocess_cfg": {"mean": OPENAI_MEAN, "std": OPENAI_STD},
}

# DFN5B-CLIP-ViT-H-14-378 (BASELINE.json configs[4]; open_clip hf-hub:apple/DFN5B-CLIP-ViT-H-14-378):
# patch 14 (K = 588), head_width 80, nn.GELU (no quick_gelu), 730 vision tokens.
VIT_H_14_378_CFG = {
    "model_cfg": {
        "embed_dim": 1024,
        "vision_cfg": {"image_size": 378, "layers": 32, "width": 1280, "head_width": 80, "patch_size": 14},
        "text_cfg": {"context_length": 77, "vocab_size": 49408, "width": 1024, "heads": 16, "layers": 24},
    },
    "preprocess_cfg": {"mean": OPENAI_MEAN, "std": OPENAI_STD},
}

# ViT-H-structured small configs: patch 14, head dim 80, erf GELU; the long one has
# 17 x 17 + 1 = 290 tokens (tiled attention, partial tiles).
TINY_H14_CFG = {
    "model_cfg": {
        "embed_dim": 64,
        "vision_cfg": {"image_size": 70, "layers": 2, "width": 320, "head_width": 80, "patch_size": 14},
        "text_cfg": {"context_length": 16, "vocab_size": 1000, "width": 128, "heads": 2, "layers": 2},
    },
    "preprocess_cfg": {"mean": OPENAI_MEAN, "std": OPENAI_STD},
}
LONG_H14_CFG = {
    "model_cfg": {
        "embed_dim": 64,
        "vision_cfg": {"image_size": 238, "layers": 2, "width": 320, "head_width": 80, "patch_size": 14},
        "text_cfg": {"context_length": 16, "vocab_size": 1000, "width": 128, "heads": 2, "layers": 2},
    },
    "preprocess_cfg": {"mean": OPENAI_MEAN, "std": OPENAI_STD},
}

# ViT-SO400M-16-SigLIP2-384 (BASELINE.json configs[3]; open_clip hf-hub:timm/ViT-SO400M-16-SigLIP2-384):
# timm trunk, 576 tokens, head dim 72, MLP 4304 (padded to 4352 on the GPU), MAP pooling.
SIGLIP_MEAN = [0.5, 0.5, 0.5]
SIGLIP_STD = [0.5, 0.5, 0.5]
SO400M_16_SIGLIP2_384_CFG = {
    "model_cfg": {
        "embed_dim": 1152,
        "init_logit_bias": -10,
        "vision_cfg": {"image_size": 384, "timm_model_name": "vit_so400m_patch16_siglip_384",
                       "timm_model_pretrained": False, "timm_pool": "map", "timm_proj": "none"},
        "text_cfg": {"context_length": 64, "vocab_size": 256000, "hf_tokenizer_name": "timm/ViT-SO400M-16-SigLIP2-384",
                     "tokenizer_kwargs": {"clean": "canonicalize"}, "width": 1152, "heads": 16, "layers": 27,
                     "mlp_ratio": 3.7362, "no_causal_mask": True, "proj_bias": True, "pool_type": "last",
                     "norm_kwargs": {"eps": 1e-6}, "act_kwargs": {"approximate": "tanh"}},
    },
    "preprocess_cfg": {"mean": SIGLIP_MEAN, "std": SIGLIP_STD, "interpolation": "bicubic", "resize_mode": "squash"},
}


def tiny_siglip_cfg(image_size=64, layers=2, mlp_width=1000):
    """SigLIP-structured synthetic config: head dim 72 (D = 576, 8 heads), MLP not a multiple of 64."""
    return {
        "model_cfg": {
            "embed_dim": 576,
            "vision_cfg": {"image_size": image_size, "timm_model_name": "vit_so400m_patch16_siglip_384",
                           "timm_pool": "map", "timm_proj": "none",
                           "clipgpu_dims": {"width": 576, "layers": layers, "heads": 8, "mlp_width": mlp_width}},
            # SigLIP2-structured text tower (head dim 72, MLP int(576 * 3.7362) = 2152, not a multiple
            # of 64, projection with bias)
            "text_cfg": {"context_length": 16, "vocab_size": 1000, "width": 576, "heads": 8, "layers": 2,
                         "mlp_ratio": 3.7362, "no_causal_mask": True, "proj_bias": True, "pool_type": "last",
                         "norm_kwargs": {"eps": 1e-6}, "act_kwargs": {"approximate": "tanh"}},
        },
        "preprocess_cfg": {"mean": SIGLIP_MEAN, "std": SIGLIP_STD},
    }


TINY_SIGLIP_CFG = tiny_siglip_cfg()
LONG_SIGLIP_CFG = tiny_siglip_cfg(image_size=384, layers=1)  # 576 tokens

# model_config.json as written by pull_onnx.py:128-150 for an OpenAI CLIP.
OPENAI_MODEL_CONFIG = {
    "logit_scale": 100.0,
    "logit_bias": 0.0,
    "activation_function": "softmax",
    "tokenizer_needs_lowercase": False,
    "pad_id": 0,
    "vocab_size": 49408,
}


def spec_dict(spec) -> dict:
    return asdict(spec)
