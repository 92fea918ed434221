"""``Clip`` facade — mirror of src/clip.rs (kept as-is in the north star; restated
here because the reference's Rust cannot be compiled in this image).  The math is
the reference's: dot -> ``mul_add(logit_scale, logit_bias)`` (defaults 1.0 / 0.0)
-> sigmoid or max-subtracted softmax -> sort descending."""
from __future__ import annotations

import math
import os
from typing import List, Sequence, Tuple

import numpy as np

from .config import ModelConfig
from .model_manager import verify_model_dir
from .text import TextEmbedder
from .vision import VisionEmbedder, _Builder


class Clip:
    def __init__(self, vision: VisionEmbedder, text: TextEmbedder, model_dir: str):
        self.vision = vision
        self.text = text
        self.model_dir = model_dir

    @classmethod
    def from_local_dir(cls, model_dir: str) -> _Builder:  # src/clip.rs:48-66
        return _Builder(cls, model_dir=model_dir)

    @classmethod
    def from_local_id(cls, model_id: str) -> _Builder:  # src/clip.rs:35-46
        return _Builder(cls, model_id=model_id)

    @classmethod
    def _build(cls, model_dir, devices, dtype, max_batch, **opts):
        verify_model_dir(model_dir, need_tokenizer=True)
        v = VisionEmbedder._build(model_dir, devices, dtype, max_batch, **opts)
        t = TextEmbedder._build(model_dir, devices, dtype, max_batch)
        return cls(v, t, model_dir)

    def duplicate(self) -> "Clip":  # src/clip.rs:68-73
        return Clip(self.vision.duplicate(), self.text.duplicate(), self.model_dir)

    def get_model_config(self) -> ModelConfig:  # src/clip.rs:75-77
        return self.text.model_config

    def _scale_bias(self):
        mc = self.text.model_config
        scale = 1.0 if mc.logit_scale is None else mc.logit_scale
        bias = 0.0 if mc.logit_bias is None else mc.logit_bias
        return np.float32(scale), np.float32(bias)

    def _activation(self) -> str:
        act = self.text.model_config.activation_function or "softmax"
        return "sigmoid" if act == "sigmoid" else "softmax"

    def _scores(self, embs: np.ndarray, query: np.ndarray, activation: str) -> np.ndarray:
        """logits = embs . query, mul_add(scale, bias), then the activation -- the reference's
        f32 arithmetic bit for bit (clipgpu_facade_scores, csrc/host/facade.cpp)."""
        from ._lib import check_host, host_lib
        from .engine import SIM_ACTIVATIONS
        e = np.ascontiguousarray(embs, dtype=np.float32)
        q = np.ascontiguousarray(query, dtype=np.float32).reshape(-1)
        if e.ndim != 2 or e.shape[1] != q.shape[0]:
            from .error import ShapeError
            raise ShapeError(f"Shape error: {e.shape} . {q.shape}")
        scale, bias = self._scale_bias()
        out = np.empty(e.shape[0], np.float32)
        check_host(host_lib().clipgpu_facade_scores(e.ctypes.data, e.shape[0], q.ctypes.data, e.shape[1],
                                                    float(scale), float(bias), SIM_ACTIVATIONS[activation],
                                                    out.ctypes.data))
        return out

    def compare(self, image, text: str) -> float:  # src/clip.rs:79-90
        v = self.vision.embed_image(image)
        t = self.text.embed_text(text)
        return float(self._scores(v[None], t, "logits")[0])

    def classify(self, image, labels: Sequence[str]) -> List[Tuple[str, float]]:  # src/clip.rs:92-132
        v = self.vision.embed_image(image)
        t = self.text.embed_texts(labels)
        probs = self._scores(t, v, self._activation())
        res = [(str(l), float(p)) for l, p in zip(labels, probs)]
        res.sort(key=lambda x: -x[1])  # stable, descending (sort_by partial_cmp)
        return res

    def rank_images(self, images, text: str) -> List[Tuple[int, float]]:  # src/clip.rs:134-170
        v = self.vision.embed_images(images)
        t = self.text.embed_text(text)
        probs = self._scores(v, t, self._activation())
        res = [(i, float(p)) for i, p in enumerate(probs)]
        res.sort(key=lambda x: -x[1])
        return res

    # -- many images x many labels, math on the GPU -------------------
    def _device_probs(self, img_embs, txt_embs, axis: int) -> np.ndarray:
        from .engine import similarity
        scale, bias = self._scale_bias()
        act = self.text.model_config.activation_function or "softmax"
        return similarity(img_embs, txt_embs, float(scale), float(bias), "sigmoid" if act == "sigmoid" else "softmax",
                          axis, self.vision.session.devices[0])

    def classify_many(self, images, labels: Sequence[str]) -> List[List[Tuple[str, float]]]:
        """classify (src/clip.rs:92-132) for every image of a batch: one image batch, one label
        batch, the [images x labels] probabilities on the GPU; each list sorted descending."""
        probs = self._device_probs(self.vision.embed_images(images), self.text.embed_texts(labels), axis=1)
        out = []
        for row in probs:
            res = [(str(l), float(p)) for l, p in zip(labels, row)]
            res.sort(key=lambda x: -x[1])
            out.append(res)
        return out

    def rank_images_many(self, images, texts: Sequence[str]) -> List[List[Tuple[int, float]]]:
        """rank_images (src/clip.rs:134-170) for every query text: softmax over the images per
        text on the GPU; one descending (image_index, probability) list per text."""
        probs = self._device_probs(self.vision.embed_images(images), self.text.embed_texts(texts), axis=0)
        out = []
        for col in probs.T:
            res = [(i, float(p)) for i, p in enumerate(col)]
            res.sort(key=lambda x: -x[1])
            out.append(res)
        return out

    @staticmethod
    def softmax(logits) -> np.ndarray:  # src/clip.rs:172-179 (f32, sequential sum; facade.cpp)
        # host-only library (no HIP / RCCL): usable on a host without ROCm
        from ._lib import check_host, host_lib
        x = np.ascontiguousarray(logits, dtype=np.float32).reshape(-1)
        if x.size == 0:
            return x.copy()
        one = np.ones(1, np.float32)  # logits = x[i] * 1 (exact) .mul_add(1, 0) (exact)
        out = np.empty(x.size, np.float32)
        check_host(host_lib().clipgpu_facade_scores(x.ctypes.data, x.size, one.ctypes.data, 1, 1.0, 0.0, 0,
                                                    out.ctypes.data))
        return out

    @staticmethod
    def sigmoid(logit: float) -> float:  # src/clip.rs:181-185
        from ._lib import check_host, host_lib
        x = np.array([logit], np.float32)
        one = np.ones(1, np.float32)
        out = np.empty(1, np.float32)
        check_host(host_lib().clipgpu_facade_scores(x.ctypes.data, 1, one.ctypes.data, 1, 1.0, 0.0, 1,
                                                    out.ctypes.data))
        return float(out[0])
