"""Model-dir contract — mirror of src/model_manager.rs.

The reference requires the nine files of ``MODEL_FILES`` (src/model_manager.rs:8-18)
because ONNX Runtime executes ``visual.onnx`` / ``text.onnx``.  The clipgpu engine
reads the same configs and tokenizer and takes its weights from, in order,
``open_clip_model.safetensors``, the initializers of ``visual.onnx`` / ``text.onnx``
(+ ``.onnx.data``; csrc/host/onnx.cpp) -- so a folder made by pull_onnx.py works as
is -- or a seeded ``clipgpu_synthetic.json``.  HF download (``get_hf_model``) is out
of scope: no network.
"""
from __future__ import annotations

import os

from .error import MissingModelFile, ModelFolderNotFound

# src/model_manager.rs:8-18 (kept for reference / ONNX-dir detection)
MODEL_FILES = [
    "model_config.json",
    "open_clip_config.json",
    "special_tokens_map.json",
    "text.onnx",
    "tokenizer.json",
    "tokenizer_config.json",
    "visual.onnx",
    "text.onnx.data",
    "visual.onnx.data",
]

CONFIG_FILES = ["model_config.json", "open_clip_config.json"]
WEIGHT_SOURCES = ["open_clip_model.safetensors", "visual.onnx", "text.onnx", "clipgpu_synthetic.json"]


def get_default_base_folder() -> str:  # src/model_manager.rs:43-49
    home = os.path.expanduser("~")
    if not home or home == "~":
        return ".open_clip_cache"
    return os.path.join(home, ".cache", "open_clip_rs")


def verify_model_dir(model_dir: str, need_tokenizer: bool = False) -> None:  # src/model_manager.rs:52-68
    if not os.path.exists(model_dir):
        raise ModelFolderNotFound(
            f"Model folder not found, generate it with `uv run pull_onnx.py -h`. '{model_dir}'")
    files = list(CONFIG_FILES) + (["tokenizer.json"] if need_tokenizer else [])
    for f in files:
        if not os.path.isfile(os.path.join(model_dir, f)):
            raise MissingModelFile(f"Missing model file '{f}' in folder '{model_dir}'")
    if not any(os.path.isfile(os.path.join(model_dir, w)) for w in WEIGHT_SOURCES):
        raise MissingModelFile(f"Missing model file 'visual.onnx' in folder '{model_dir}'")
