"""Pin the oracle (oracle/clip_ref.py, fp64 restatement of the exported graphs) against
(a) the committed golden embeddings (regression) and (b) HF transformers CLIP towers
loaded with the same weights — an independent implementation of the same architecture
(the reference's own ONNX/open_clip path cannot run offline)."""
import os

import numpy as np
import pytest

from oracle import clip_ref, weights
from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, TINY_CFG, VIT_B_32_CFG, text_spec_from_cfg, \
    vision_spec_from_cfg

GOLD = os.path.join(os.path.dirname(__file__), "golden", "embed_golden.npz")


def pixels(v, B):
    u8 = weights.synth_images_u8(100, B, v.image_size)
    return ((u8.astype(np.float32) / np.float32(255) - np.asarray(OPENAI_MEAN, np.float32))
            / np.asarray(OPENAI_STD, np.float32)).transpose(0, 3, 1, 2)


@pytest.mark.parametrize("name,cfg,B", [("tiny", TINY_CFG, 3), ("b32", VIT_B_32_CFG, 2)])
def test_oracle_matches_golden_and_hf(name, cfg, B):
    g = np.load(GOLD)
    v, t = vision_spec_from_cfg(cfg["model_cfg"]), text_spec_from_cfg(cfg["model_cfg"])
    ov = clip_ref.encode_image(weights.vision_weights(v, 1234), v, pixels(v, B))
    assert np.allclose(ov, g[f"{name}_vision_oracle"], atol=1e-12)
    assert clip_ref.cosine_rows(g[f"{name}_vision_oracle"], g[f"{name}_vision_hf"]).min() > 1 - 1e-9
    ids = g[f"{name}_text_ids"]
    ot = clip_ref.encode_text(weights.text_weights(t, 1234), t, ids)
    assert np.allclose(ot, g[f"{name}_text_oracle"], atol=1e-12)
    assert clip_ref.cosine_rows(g[f"{name}_text_oracle"], g[f"{name}_text_hf"]).min() > 1 - 1e-9


@pytest.mark.parametrize("cfg_name", ["TINY_CFG", "TINY_H14_CFG", "LONG_H14_CFG"])
def test_oracle_vs_hf_live_tiny(cfg_name):
    """Also the ViT-H/14 structure (patch 14, head dim 80, erf GELU, 290 tokens)."""
    pytest.importorskip("transformers")
    from oracle import hf_pin, model_spec
    cfg = getattr(model_spec, cfg_name)
    v, t = vision_spec_from_cfg(cfg["model_cfg"]), text_spec_from_cfg(cfg["model_cfg"])
    P = weights.vision_weights(v, 99)
    px = pixels(v, 2)
    assert np.abs(clip_ref.encode_image(P, v, px) - hf_pin.hf_encode_image(hf_pin.hf_vision(P, v), px)).max() < 1e-7
    PT = weights.text_weights(t, 99)
    ids = weights.synth_token_ids(5, 3, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                  random_eot=True)
    assert np.abs(clip_ref.encode_text(PT, t, ids) - hf_pin.hf_encode_text(hf_pin.hf_text(PT, t), ids)).max() < 1e-7


def test_oracle_properties():
    v, t = vision_spec_from_cfg(TINY_CFG["model_cfg"]), text_spec_from_cfg(TINY_CFG["model_cfg"])
    P = weights.vision_weights(v, 3)
    px = pixels(v, 3)
    e = clip_ref.encode_image(P, v, px)
    assert np.allclose(np.linalg.norm(e, axis=1), 1)
    # batch independence: rows do not interact
    assert np.allclose(clip_ref.encode_image(P, v, px[1:2]), e[1:2], atol=1e-12)
    # text: tokens after the first EOT do not change the output
    PT = weights.text_weights(t, 3)
    ids = weights.synth_token_ids(8, 2, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                  random_eot=True)
    ids2 = ids.copy()
    p = int(np.argmax(ids2[0]))
    ids2[0, p + 1:] = 7
    assert np.allclose(clip_ref.encode_text(PT, t, ids)[0], clip_ref.encode_text(PT, t, ids2)[0], atol=1e-12)


@pytest.mark.parametrize("cfg_name", ["TINY_SIGLIP_CFG", "LONG_SIGLIP_CFG"])
def test_siglip_oracle_vs_hf(cfg_name):
    """SigLIP family (timm trunk + MAP head, BASELINE configs[3] structure) vs HF SiglipVisionModel."""
    pytest.importorskip("transformers")
    from oracle import hf_pin, model_spec
    cfg = getattr(model_spec, cfg_name)
    v = vision_spec_from_cfg(cfg["model_cfg"])
    assert v.family == "siglip" and v.head_dim == 72 and v.tokens == v.grid ** 2
    P = weights.vision_weights(v, 5)
    px = pixels(v, 2)
    got = clip_ref.encode_image(P, v, px)
    ref = hf_pin.hf_siglip_encode_image(hf_pin.hf_siglip_vision(P, v), px)
    assert np.abs(got - ref).max() < 1e-7


@pytest.mark.parametrize("ctx,layers", [(16, 2), (64, 1)])
def test_siglip2_text_oracle_vs_hf(ctx, layers):
    """SigLIP2-form text tower (open_clip text_cfg no_causal_mask, pool_type "last", proj_bias,
    GELU tanh, eps 1e-6; head dim 72, MLP 2152) vs HF SiglipTextModel on the same weights: no
    causal mask, the last context position pooled (padding included), `head` Linear with bias."""
    pytest.importorskip("transformers")
    from oracle import hf_pin, model_spec
    cfg = model_spec.tiny_siglip_cfg()
    cfg["model_cfg"]["text_cfg"].update({"context_length": ctx, "layers": layers})
    t = text_spec_from_cfg(cfg["model_cfg"])
    assert (not t.causal, t.pool, t.proj_bias, t.act, t.ln_eps, t.head_dim, t.mlp_width) == \
        (True, "last", True, "gelu_tanh", 1e-6, 72, 2152)
    P = weights.text_weights(t, 11)
    ids = weights.synth_token_ids(6, 3, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                  random_eot=True)
    got = clip_ref.encode_text(P, t, ids)
    assert np.abs(got - hf_pin.hf_siglip_encode_text(hf_pin.hf_siglip_text(P, t), ids)).max() < 1e-7
    # every position reaches the pooled (last) one: a token after the "EOT" changes the output
    ids2 = ids.copy()
    p = int(np.argmax(ids2[0]))
    ids2[0, p + 1:] = 7
    assert clip_ref.cosine_rows(clip_ref.encode_text(P, t, ids2)[:1], got[:1]).min() < 1 - 1e-9


def test_so400m_siglip2_text_spec():
    from oracle import model_spec
    t = text_spec_from_cfg(model_spec.SO400M_16_SIGLIP2_384_CFG["model_cfg"])
    assert (t.context_length, t.vocab_size, t.width, t.layers, t.heads, t.mlp_width, t.embed_dim, t.head_dim) == \
        (64, 256000, 1152, 27, 16, 4304, 1152, 72)
    assert (t.causal, t.pool, t.proj_bias, t.act, t.ln_eps) == (False, "last", True, "gelu_tanh", 1e-6)


def test_so400m_siglip2_spec():
    from oracle import model_spec
    v = vision_spec_from_cfg(model_spec.SO400M_16_SIGLIP2_384_CFG["model_cfg"])
    assert (v.patch_size, v.width, v.layers, v.heads, v.mlp_width, v.tokens, v.head_dim) == \
        (16, 1152, 27, 16, 4304, 576, 72)
    assert v.act == "gelu_tanh" and v.ln_eps == 1e-6 and v.embed_dim == 1152


@pytest.mark.parametrize("cfg_name", ["TINY_CFG", "VIT_B_32_CFG", "TINY_SIGLIP_CFG"])
def test_torch_cpu_port_matches_oracle(cfg_name):
    """oracle/torch_cpu.py (the fp32 CPU baseline bench.py times) computes the fp64 oracle's
    embeddings to fp32 accuracy."""
    from oracle import model_spec, torch_cpu
    from oracle.model_spec import text_spec_from_cfg, vision_spec_from_cfg
    cfg = getattr(model_spec, cfg_name)
    v = vision_spec_from_cfg(cfg["model_cfg"])
    t = text_spec_from_cfg(cfg["model_cfg"])
    Pv = weights.vision_weights(v, 5)
    Pt = weights.text_weights(t, 5)
    px = np.random.default_rng(3).standard_normal((2, 3, v.image_size, v.image_size)).astype(np.float32)
    ids = weights.synth_token_ids(4, 3, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                  random_eot=True)
    cv = (clip_ref.cosine_rows(torch_cpu.VisionCPU(Pv, v)(px), clip_ref.encode_image(Pv, v, px))
          if v.family == "clip" else np.ones(1))  # SigLIP vision: the MAP head is not ported
    ct = clip_ref.cosine_rows(torch_cpu.TextCPU(Pt, t)(ids), clip_ref.encode_text(Pt, t, ids))
    assert cv.min() > 0.999999 and ct.min() > 0.999999, (cv, ct)


def test_layernorm_fold_identity():
    """The algebra behind the engine's LayerNorm fold (EPI_LNF): for a Linear
    W, b behind LayerNorm (gamma, beta), LN(x) W^T + b = rstd (x W'^T - mean cs) + (b + W beta) with
    W' = W diag(gamma), cs = W' 1, mean / rstd of each row of x.  Checked in fp64 on the oracle's
    own LayerNorm (`clip_ref.layer_norm`) and on residual-stream-like rows (per-row offsets, a few
    massive channels), then with W' rounded to f16 and x in f16 as the GPU computes it: the
    difference stays far inside the bf16 output rounding."""
    rng = np.random.default_rng(3)
    M, K, N = 64, 768, 256
    x = rng.standard_normal((M, K)) * rng.uniform(0.5, 4.0, (M, 1)) + rng.standard_normal((M, 1))
    x[:, [7, 300, 511]] *= 40.0
    w = rng.standard_normal((N, K)) / np.sqrt(K)
    g, beta, b = 1 + 0.2 * rng.standard_normal(K), 0.1 * rng.standard_normal(K), 0.1 * rng.standard_normal(N)
    ref = clip_ref.layer_norm(x, g, beta, 1e-5) @ w.T + b
    mean = x.mean(1, keepdims=True)
    rstd = 1.0 / np.sqrt(((x - mean) ** 2).mean(1, keepdims=True) + 1e-5)
    wf = w * g
    fold = rstd * (x @ wf.T - mean * wf.sum(1)) + (b + w @ beta)
    assert np.abs(fold - ref).max() <= 1e-9 * np.abs(ref).max()
    # the GPU's operand rounding: x (the stream) and W' in f16
    x16, wf16 = x.astype(np.float16).astype(np.float64), wf.astype(np.float16).astype(np.float64)
    mean16 = x16.mean(1, keepdims=True)
    rstd16 = 1.0 / np.sqrt(((x16 - mean16) ** 2).mean(1, keepdims=True) + 1e-5)
    gpu = rstd16 * (x16 @ wf16.T - mean16 * wf16.sum(1)) + (b + w @ beta)
    assert np.abs(gpu - ref).max() <= 2.0 ** -9 * np.sqrt((ref ** 2).mean()) * 4
