"""Error type mirroring ``ClipError`` (src/error.rs:9-41).

The C ABI returns a status code (include/clipgpu.h ``clipgpu_status``) plus a
thread-local message; ``error_for_status`` maps it onto the reference's variants.
"""
from __future__ import annotations


class ClipError(Exception):
    """Base error (``ClipError``)."""


class IoError(ClipError):
    """``ClipError::Io``"""


class ConfigError(ClipError):
    """``ClipError::Config`` / ``ModelFolderNotFound`` / ``MissingModelFile``"""


class InferenceError(ClipError):
    """``ClipError::Inference`` (e.g. "Empty batch", src/vision.rs:121-123)"""


class ShapeError(ClipError):
    """``ClipError::Shape``"""


class TokenizerError(ClipError):
    """``ClipError::Tokenizer``"""


class ModelFolderNotFound(ConfigError):
    """``ClipError::ModelFolderNotFound`` (src/error.rs:29-30)"""


class MissingModelFile(ConfigError):
    """``ClipError::MissingModelFile`` (src/error.rs:34-35)"""


def error_for_status(code: int, msg: str) -> ClipError:
    if code == 2:
        if msg.startswith("Model folder not found"):
            return ModelFolderNotFound(msg)
        if msg.startswith("Missing model file"):
            return MissingModelFile(msg)
        return ConfigError(msg)
    if code == 3:
        return IoError(msg)
    if code == 5:
        return TokenizerError(msg)
    if code == 1 and msg.startswith("Shape error"):
        return ShapeError(msg)
    return InferenceError(msg)
