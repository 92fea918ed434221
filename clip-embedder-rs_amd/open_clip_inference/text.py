"""``TextEmbedder`` — drop-in mirror of src/text.rs.

Tokenisation runs in the native CLIP BPE tokenizer (csrc/host/tokenizer.cpp),
the forward pass in the HIP engine.
"""
from __future__ import annotations

import os
from typing import Sequence

import numpy as np

from . import _lib
from .config import ModelConfig, OpenClipConfig
from .engine import Engine, Tokenizer
from .error import ConfigError, InferenceError
from .model_manager import verify_model_dir
from .vision import _Builder


class TextEmbedder:
    def __init__(self, engine: Engine, config: OpenClipConfig, model_config: ModelConfig, model_dir: str,
                 tokenizer: Tokenizer):
        self.session = engine
        self.config = config
        self.model_config = model_config
        self.model_dir = model_dir
        self._tokenizer = tokenizer
        self._id_name = "input_ids"
        self._mask_name = None  # the exported text graph has no mask input (pull_onnx.py:296-302)

    @classmethod
    def from_local_dir(cls, model_dir: str) -> _Builder:
        return _Builder(cls, model_dir=model_dir)

    @classmethod
    def from_local_id(cls, model_id: str) -> _Builder:
        return _Builder(cls, model_id=model_id)

    @classmethod
    def _build(cls, model_dir, devices, dtype, max_batch, engine_opts=None, **_opts):  # src/text.rs:54-101
        verify_model_dir(model_dir, need_tokenizer=True)
        model_config = ModelConfig.from_file(os.path.join(model_dir, "model_config.json"))
        config = OpenClipConfig.from_file(os.path.join(model_dir, "open_clip_config.json"))
        ctx = config.model_cfg.text_cfg.context_length
        tok = Tokenizer(os.path.join(model_dir, "tokenizer.json"), ctx, model_config.pad_id)
        engine = Engine(model_dir, _lib.TOWER_TEXT, devices, dtype, max_batch or 1024, **(engine_opts or {}))
        return cls(engine, config, model_config, model_dir, tok)

    def duplicate(self) -> "TextEmbedder":  # src/text.rs:103-108
        e = self.session
        return self._build(self.model_dir, e.devices, e.dtype, e.max_batch, e.opts)

    def tokenize(self, texts: Sequence[str]):  # src/text.rs:110-139
        return self._tokenizer.encode_batch(list(texts), lowercase=self.model_config.tokenizer_needs_lowercase)

    def embed_text(self, text: str) -> np.ndarray:  # src/text.rs:141-146
        return self.embed_texts([text]).reshape(-1)

    def embed_texts(self, texts: Sequence[str]) -> np.ndarray:  # src/text.rs:148-169
        if len(texts) == 0:
            raise InferenceError("Empty batch")
        ids, mask = self.tokenize(texts)
        return self.session.embed_tokens(ids, mask)
