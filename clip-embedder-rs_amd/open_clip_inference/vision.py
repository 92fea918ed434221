"""``VisionEmbedder`` — drop-in mirror of src/vision.rs.

Preprocessing (crop/resize/normalise) runs in the native host library
(csrc/host/preprocess.cpp), the forward pass in the HIP engine.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .config import ModelConfig, OpenClipConfig
from .engine import Engine, preprocess_batch_rgb8
from .error import InferenceError
from .model_manager import get_default_base_folder, verify_model_dir


def to_rgb8(image) -> np.ndarray:
    """``DynamicImage::to_rgb8`` for PIL images or HxWx3 / HxW uint8 arrays."""
    if hasattr(image, "convert") and hasattr(image, "size"):  # PIL.Image
        image = np.asarray(image.convert("RGB"))
    a = np.asarray(image)
    if a.ndim == 2:
        a = np.repeat(a[:, :, None], 3, axis=2)
    if a.ndim != 3 or a.shape[2] not in (3, 4):
        raise InferenceError(f"unsupported image shape {a.shape}")
    return np.ascontiguousarray(a[:, :, :3], dtype=np.uint8)


class _Builder:
    """bon-style builder: ``X.from_local_dir(p).with_devices([0]).build()``."""

    def __init__(self, cls, model_dir: Optional[str] = None, model_id: Optional[str] = None):
        self._cls = cls
        self._model_dir = model_dir
        self._model_id = model_id
        self._base = None
        self._devices = None
        self._dtype = "bf16"
        self._max_batch = None
        self._opts = {}
        self._engine = {}

    def base_folder(self, path: str):
        self._base = path
        return self

    def with_devices(self, devices: Sequence[int]):  # replaces with_execution_providers
        self._devices = list(devices)
        return self

    def with_dtype(self, dtype: str):
        self._dtype = dtype
        return self

    def with_max_batch(self, n: int):
        self._max_batch = int(n)
        return self

    def with_mx_sites(self, sites):
        """fp8 engines: the GEMM sites that run MX-fp8 ("qkv", "fc", "proj"; default all three),
        per engine (clipgpu_options.mx_sites)."""
        self._engine["mx_sites"] = sites
        return self

    def with_lanes(self, lanes: int):
        """Concurrent sub-batch lanes per device (clipgpu_options.lanes; 0 = the tile table's)."""
        self._engine["lanes"] = int(lanes)
        return self

    def with_resize_impl(self, impl: str):
        """The resize the crate's `fast_image_resize` feature selects (src/vision.rs:149-157):
        "fast_image_resize" (default feature) or "image" (resize_with_image, :200-233)."""
        from .engine import RESIZE_IMPLS
        if impl not in RESIZE_IMPLS:
            raise ValueError(f"resize impl must be one of {RESIZE_IMPLS}")
        self._opts["resize_impl"] = impl
        return self

    def build(self):
        d = self._model_dir
        if d is None:
            d = os.path.join(self._base or get_default_base_folder(), self._model_id)
        return self._cls._build(d, self._devices, self._dtype, self._max_batch, engine_opts=dict(self._engine),
                                **self._opts)


class VisionEmbedder:
    def __init__(self, engine: Engine, config: OpenClipConfig, model_config: ModelConfig, model_dir: str,
                 resize_impl: str = "fast_image_resize"):
        self.session = engine          # pub session (src/vision.rs:21) -> engine handle
        self.config = config
        self.model_config = model_config
        self.input_name = "pixel_values"
        self.model_dir = model_dir
        self.resize_impl = resize_impl

    # -- builders (src/vision.rs:45-84) --
    @classmethod
    def from_local_dir(cls, model_dir: str) -> _Builder:
        return _Builder(cls, model_dir=model_dir)

    @classmethod
    def from_local_id(cls, model_id: str) -> _Builder:
        return _Builder(cls, model_id=model_id)

    @classmethod
    def _build(cls, model_dir, devices, dtype, max_batch, resize_impl="fast_image_resize", engine_opts=None):
        verify_model_dir(model_dir)
        config = OpenClipConfig.from_file(os.path.join(model_dir, "open_clip_config.json"))
        model_config = ModelConfig.from_file(os.path.join(model_dir, "model_config.json"))
        engine = Engine(model_dir, _lib.TOWER_VISION, devices, dtype, max_batch or 256, **(engine_opts or {}))
        return cls(engine, config, model_config, model_dir, resize_impl)

    def duplicate(self) -> "VisionEmbedder":  # src/vision.rs:86-91
        e = self.session
        return self._build(self.model_dir, e.devices, e.dtype, e.max_batch, self.resize_impl, e.opts)

    # -- embedding (src/vision.rs:93-117) --
    def embed_image(self, image) -> np.ndarray:
        embs = self.embed_images([image])
        return embs.reshape(-1)

    def embed_images(self, images) -> np.ndarray:
        # preprocess_batch + run (src/vision.rs:100-117), with the crop/resize/normalise on the
        # GPU: bit-identical to self.session.embed_pixels(self.preprocess_batch(images)).
        if len(images) == 0:
            raise InferenceError("Empty batch")
        if self.resize_impl == "image":  # resize_with_image runs on the host (no GPU form)
            return self.session.embed_pixels(self.preprocess_batch(images))
        return self.session.embed_images_rgb8([to_rgb8(im) for im in images])

    # -- preprocessing (src/vision.rs:119-140) --
    def preprocess_batch(self, images) -> np.ndarray:
        if len(images) == 0:
            raise InferenceError("Empty batch")
        pc = self.config.preprocess_cfg
        size = self.config.model_cfg.vision_cfg.image_size
        return preprocess_batch_rgb8([to_rgb8(im) for im in images], size, pc.interpolation, pc.resize_mode,
                                     pc.mean, pc.std, self.resize_impl)

    def preprocess(self, image) -> np.ndarray:
        return self.preprocess_batch([image])
