"""``ModelConfig`` / ``OpenClipConfig`` — mirror of src/config.rs:6-71.

The C++ engine parses the same files itself (csrc/host/config.cpp); this mirror
exists so that callers see the same fields the reference exposes
(``VisionEmbedder.config`` / ``.model_config``, src/vision.rs:20-27).
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class ModelConfig:  # src/config.rs:6-14
    tokenizer_needs_lowercase: bool = False
    activation_function: Optional[str] = None
    logit_scale: Optional[float] = None
    logit_bias: Optional[float] = None
    pad_id: Optional[int] = None

    @classmethod
    def from_file(cls, path: str) -> "ModelConfig":  # src/config.rs:16-21
        with open(path) as f:
            d = json.load(f)
        return cls(
            tokenizer_needs_lowercase=bool(d.get("tokenizer_needs_lowercase", False)),
            activation_function=d.get("activation_function"),
            logit_scale=d.get("logit_scale"),
            logit_bias=d.get("logit_bias"),
            pad_id=d.get("pad_id"),
        )


@dataclass
class VisionCfg:  # src/config.rs:36-41
    image_size: int
    layers: Optional[int] = None
    width: Optional[int] = None


@dataclass
class TextCfg:  # src/config.rs:43-47
    context_length: int
    hf_tokenizer_name: Optional[str] = None


@dataclass
class ModelCfg:  # src/config.rs:29-34
    embed_dim: int
    vision_cfg: VisionCfg
    text_cfg: TextCfg


@dataclass
class PreprocessCfg:  # src/config.rs:49-64
    mean: List[float]
    std: List[float]
    interpolation: str = "bicubic"
    resize_mode: str = "shortest"


@dataclass
class OpenClipConfig:  # src/config.rs:23-27
    model_cfg: ModelCfg
    preprocess_cfg: PreprocessCfg
    raw: dict = field(default_factory=dict, repr=False)

    @classmethod
    def from_file(cls, path: str) -> "OpenClipConfig":  # src/config.rs:66-71
        with open(path) as f:
            d = json.load(f)
        mc = d["model_cfg"]
        v = mc["vision_cfg"]
        t = mc["text_cfg"]
        p = d["preprocess_cfg"]
        return cls(
            model_cfg=ModelCfg(
                embed_dim=int(mc["embed_dim"]),
                vision_cfg=VisionCfg(int(v["image_size"]), v.get("layers"), v.get("width")),
                text_cfg=TextCfg(int(t["context_length"]), t.get("hf_tokenizer_name")),
            ),
            preprocess_cfg=PreprocessCfg(
                mean=[float(x) for x in p["mean"]],
                std=[float(x) for x in p["std"]],
                interpolation=p.get("interpolation", "bicubic"),
                resize_mode=p.get("resize_mode", "shortest"),
            ),
            raw=d,
        )
