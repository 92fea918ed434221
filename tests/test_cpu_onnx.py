"""ONNX weight ingestion (csrc/host/onnx.cpp) -- the reference's own model-folder format.

Model folders are exported the way pull_onnx.py:170-195 does it (tests/onnx_export.py:
open_clip-structured torch towers, torch.onnx.export with the same arguments), so the
files carry a real exporter's initializer names, constant-folded (pre-transposed,
anonymous "onnx::MatMul_N") linear weights and de-duplicated tensors.  Bar: every
parameter read back bit-exact (f32 export) with and without external .onnx.data.
The torch forward of the same towers also pins the oracle (cos >= 1 - 1e-6).
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from oracle import clip_ref, weights
from oracle.model_spec import OPENAI_MEAN, OPENAI_MODEL_CONFIG, OPENAI_STD, TINY_CFG
from tests.helpers import normalized_pixels, specs
from tests.onnx_export import export_model_dir, initializer_names


def _onnx_dir(tmp_path, external):
    d = tmp_path / ("ext" if external else "inline")
    d.mkdir()
    with open(d / "open_clip_config.json", "w") as f:
        json.dump(TINY_CFG, f)
    with open(d / "model_config.json", "w") as f:
        json.dump(OPENAI_MODEL_CONFIG, f)
    v, t = specs(TINY_CFG)
    model = export_model_dir(str(d), v, t, seed=77, external=external)
    return str(d), model


def _read(d, tower, name, shape):
    from open_clip_inference import _lib
    out = np.empty(int(np.prod(shape)), np.float32)
    _lib.check(_lib.lib().clipgpu_test_read_weights(d.encode(), tower, name.encode(), out.ctypes.data, out.size))
    return out.reshape(shape)


@pytest.mark.parametrize("external", [False, True])
def test_onnx_weights_bit_exact(tmp_path, external):
    d, _ = _onnx_dir(tmp_path, external)
    names = initializer_names(os.path.join(d, "visual.onnx"))
    # the real exporter folded the linear weights into anonymous transposed initializers
    assert any(n.startswith("onnx::MatMul") for n in names), names
    assert "model.visual.conv1.weight" in names
    if external:
        assert os.path.getsize(os.path.join(d, "visual.onnx.data")) > 0
    v, t = specs(TINY_CFG)
    for tower, P in ((0, weights.vision_weights(v, 77)), (1, weights.text_weights(t, 77))):
        for name, ref in P.items():
            got = _read(d, tower, name, ref.shape)
            assert np.array_equal(got, ref.astype(np.float32)), name


def test_torch_towers_pin_oracle(tmp_path):
    """The exported torch towers (nn.MultiheadAttention etc.) agree with oracle/clip_ref.py."""
    v, t = specs(TINY_CFG)
    from tests.onnx_export import build_model
    m = build_model(v, t, seed=77)
    u8 = weights.synth_images_u8(5, 3, v.image_size)
    px = normalized_pixels(u8, OPENAI_MEAN, OPENAI_STD)
    with torch.no_grad():
        got = m.encode_image(torch.from_numpy(px), normalize=True).double().numpy()
    ref = clip_ref.encode_image(weights.vision_weights(v, 77), v, px)
    assert clip_ref.cosine_rows(got, ref).min() > 1 - 1e-6
    ids = weights.synth_token_ids(6, 4, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                  random_eot=True)
    with torch.no_grad():
        got = m.encode_text(torch.from_numpy(ids), normalize=True).double().numpy()
    ref = clip_ref.encode_text(weights.text_weights(t, 77), t, ids)
    assert clip_ref.cosine_rows(got, ref).min() > 1 - 1e-6


def test_onnx_missing_tensor_error(tmp_path):
    from open_clip_inference import _lib
    from open_clip_inference.error import ClipError
    d = tmp_path / "bad"
    d.mkdir()
    cfg = json.loads(json.dumps(TINY_CFG))
    cfg["model_cfg"]["vision_cfg"]["layers"] = 3  # the export has 2 blocks
    v, t = specs(TINY_CFG)
    export_model_dir(str(d), v, t, seed=1)
    with open(d / "open_clip_config.json", "w") as f:
        json.dump(cfg, f)
    out = np.empty(4, np.float32)
    with pytest.raises(ClipError, match="resblocks.2"):
        _lib.check(_lib.lib().clipgpu_test_read_weights(str(d).encode(), 0,
                                                        b"visual.transformer.resblocks.2.ln_1.weight",
                                                        out.ctypes.data, 4))


@pytest.mark.parametrize("external", [False, True])
def test_onnx_siglip_weights_bit_exact(tmp_path, external):
    """SigLIP family (timm trunk names): folded qkv/proj/fc1/fc2/q/kv MatMul weights, pos_embed,
    attn_pool latent, through a real torch.onnx.export of the restated timm module tree."""
    from oracle.model_spec import TINY_SIGLIP_CFG
    from tests.onnx_export import build_siglip_vision, export_siglip_visual
    d = tmp_path / "siglip"
    d.mkdir()
    with open(d / "open_clip_config.json", "w") as f:
        json.dump(TINY_SIGLIP_CFG, f)
    with open(d / "model_config.json", "w") as f:
        json.dump(OPENAI_MODEL_CONFIG, f)
    v, _ = specs(TINY_SIGLIP_CFG)
    export_siglip_visual(str(d), v, seed=78, external=external)
    names = initializer_names(os.path.join(d, "visual.onnx"))
    assert any(n.startswith("onnx::MatMul") for n in names), names
    for name, ref in weights.vision_weights(v, 78).items():
        got = _read(str(d), 0, name, ref.shape)
        assert np.array_equal(got, ref.astype(np.float32)), name
    # the restated timm module tree also pins the oracle
    m = build_siglip_vision(v, 78)
    px = normalized_pixels(weights.synth_images_u8(5, 2, v.image_size), [0.5] * 3, [0.5] * 3)
    with torch.no_grad():
        got = m.encode_image(torch.from_numpy(px), normalize=True).double().numpy()
    ref = clip_ref.encode_image(weights.vision_weights(v, 78), v, px)
    assert clip_ref.cosine_rows(got, ref).min() > 1 - 1e-6


@pytest.mark.parametrize("external", [False, True])
def test_onnx_siglip2_text_weights_bit_exact(tmp_path, external):
    """SigLIP2 text tower (no causal mask, last-position pooling, nn.Linear projection with bias):
    every parameter of a real torch.onnx.export of the restated open_clip TextTransformer read back
    bit-exact (the folded text_projection MatMul and its bias included); the torch tower pins the
    oracle."""
    from oracle.model_spec import TINY_SIGLIP_CFG
    from tests.onnx_export import export_siglip_text
    d = tmp_path / "siglip_text"
    d.mkdir()
    with open(d / "open_clip_config.json", "w") as f:
        json.dump(TINY_SIGLIP_CFG, f)
    with open(d / "model_config.json", "w") as f:
        json.dump(OPENAI_MODEL_CONFIG, f)
    _, t = specs(TINY_SIGLIP_CFG)
    m = export_siglip_text(str(d), t, seed=79, external=external)
    P = weights.text_weights(t, 79)
    for name, ref in P.items():
        got = _read(str(d), 1, name, ref.shape)
        assert np.array_equal(got, ref.astype(np.float32)), name
    ids = weights.synth_token_ids(6, 3, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                  random_eot=True)
    with torch.no_grad():
        got = m.encode_text(torch.from_numpy(ids), normalize=True).double().numpy()
    assert clip_ref.cosine_rows(got, clip_ref.encode_text(P, t, ids)).min() > 1 - 1e-6
