"""open_clip_inference — MI355X-native drop-in for the crate of the same name
(RuurdBijlsma/clip-embedder-rs v0.4.0, src/lib.rs:170-181 re-exports).

Host API mirror in Python over the clipgpu C ABI (include/clipgpu.h).  The compute
runs in ``lib/libclipgpu.so`` (hand-written gfx950 HIP kernels + C++ host runtime).
"""
from .clip import Clip
from .config import ModelConfig, OpenClipConfig
from .error import ClipError
from .text import TextEmbedder
from .vision import VisionEmbedder

__all__ = ["Clip", "ClipError", "TextEmbedder", "VisionEmbedder", "ModelConfig", "OpenClipConfig"]
