"""fp32 CPU port of the reference's graphs on torch — TEST / BASELINE INFRASTRUCTURE.

The CPU baseline `bench.py` times beside the GPU value (its `cpu_baseline` leg only).  The
reference runs `visual.onnx` / `text.onnx` on ONNX Runtime's CPU provider (MLAS sgemm,
`intra_threads = num_cpus::get()`, src/onnx.rs:18-22); neither ORT nor the Rust toolchain is in
this image, so this is the closest proxy buildable here: the same graph arithmetic as
`oracle/clip_ref.py` (open_clip encode_image / encode_text with normalize=True,
pull_onnx.py:53-68) in fp32 on torch's CPU kernels (oneDNN / MKL sgemm, fused CPU attention), all
host threads torch is given.  Pinned to clip_ref at fp32 tolerance by
tests/test_cpu_oracle.py::test_torch_cpu_port_matches_oracle.  CLIP family only (the bench model).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

from .model_spec import TextSpec, VisionSpec


def _act(name, x):
    if name == "quick_gelu":
        return x * torch.sigmoid(1.702 * x)
    if name == "gelu":
        return F.gelu(x)
    if name == "gelu_tanh":
        return F.gelu(x, approximate="tanh")
    raise ValueError(name)


class _Tower:
    def __init__(self, P: Dict[str, np.ndarray], prefix: str, layers: int, heads: int, width: int, act: str,
                 eps: float):
        self.heads, self.width, self.act, self.eps = heads, width, act, eps
        t = lambda k: torch.from_numpy(np.ascontiguousarray(P[k], np.float32))  # noqa: E731
        self.blocks = []
        for i in range(layers):
            p = f"{prefix}{i}."
            self.blocks.append({
                "ln1": (t(p + "ln_1.weight"), t(p + "ln_1.bias")),
                "qkv": (t(p + "attn.in_proj_weight"), t(p + "attn.in_proj_bias")),
                "out": (t(p + "attn.out_proj.weight"), t(p + "attn.out_proj.bias")),
                "ln2": (t(p + "ln_2.weight"), t(p + "ln_2.bias")),
                "fc": (t(p + "mlp.c_fc.weight"), t(p + "mlp.c_fc.bias")),
                "proj": (t(p + "mlp.c_proj.weight"), t(p + "mlp.c_proj.bias")),
            })

    def __call__(self, x, causal):
        B, N, D = x.shape
        H = self.heads
        for b in self.blocks:
            h = F.layer_norm(x, (D,), *b["ln1"], self.eps)
            qkv = F.linear(h, *b["qkv"]).view(B, N, 3, H, D // H).permute(2, 0, 3, 1, 4)
            o = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2], is_causal=causal)
            x = x + F.linear(o.transpose(1, 2).reshape(B, N, D), *b["out"])
            h = F.layer_norm(x, (D,), *b["ln2"], self.eps)
            x = x + F.linear(_act(self.act, F.linear(h, *b["fc"])), *b["proj"])
        return x


class VisionCPU:
    """open_clip VisionTransformer.forward + F.normalize, fp32 on the CPU."""

    def __init__(self, P: Dict[str, np.ndarray], v: VisionSpec):
        assert v.family != "siglip", "CLIP family only"
        self.v = v
        t = lambda k: torch.from_numpy(np.ascontiguousarray(P[k], np.float32))  # noqa: E731
        self.conv = t("visual.conv1.weight")
        self.cls, self.pos = t("visual.class_embedding"), t("visual.positional_embedding")
        self.ln_pre = (t("visual.ln_pre.weight"), t("visual.ln_pre.bias"))
        self.ln_post = (t("visual.ln_post.weight"), t("visual.ln_post.bias"))
        self.proj = t("visual.proj")
        self.trunk = _Tower(P, "visual.transformer.resblocks.", v.layers, v.heads, v.width, v.act, v.ln_eps)

    @torch.inference_mode()
    def __call__(self, pixels: np.ndarray) -> np.ndarray:
        v = self.v
        x = torch.from_numpy(np.ascontiguousarray(pixels, np.float32))
        B, D = x.shape[0], v.width
        x = F.conv2d(x, self.conv, stride=v.patch_size).flatten(2).transpose(1, 2)
        x = torch.cat([self.cls.expand(B, 1, D), x], 1) + self.pos
        x = F.layer_norm(x, (D,), *self.ln_pre, v.ln_eps)
        x = self.trunk(x, causal=False)
        x = F.layer_norm(x[:, 0], (D,), *self.ln_post, v.ln_eps) @ self.proj
        return F.normalize(x, dim=-1).numpy()


class TextCPU:
    """open_clip encode_text + F.normalize, fp32 on the CPU: CLIP (causal, argmax / EOT pooling,
    projection matrix) or SigLIP2 (no mask, last-position pooling, linear projection with bias)."""

    def __init__(self, P: Dict[str, np.ndarray], t: TextSpec):
        self.t = t
        tt = lambda k: torch.from_numpy(np.ascontiguousarray(P[k], np.float32))  # noqa: E731
        self.tok, self.pos = tt("token_embedding.weight"), tt("positional_embedding")
        self.ln_final = (tt("ln_final.weight"), tt("ln_final.bias"))
        if t.proj_bias:
            self.proj, self.proj_b = tt("text_projection.weight").T.contiguous(), tt("text_projection.bias")
        else:
            self.proj, self.proj_b = tt("text_projection"), None
        self.trunk = _Tower(P, "transformer.resblocks.", t.layers, t.heads, t.width, t.act, t.ln_eps)

    @torch.inference_mode()
    def __call__(self, ids: np.ndarray) -> np.ndarray:
        ids = torch.from_numpy(np.ascontiguousarray(ids, np.int64))
        B, T = ids.shape
        x = self.tok[ids] + self.pos[:T]
        x = self.trunk(x, causal=self.t.causal)
        pooled = x[:, -1] if self.t.pool == "last" else x[torch.arange(B), ids.argmax(-1)]
        x = F.layer_norm(pooled, (self.t.width,), *self.ln_final, self.t.ln_eps)
        y = x @ self.proj
        if self.proj_b is not None:
            y = y + self.proj_b
        return F.normalize(y, dim=-1).numpy()
