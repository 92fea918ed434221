"""MX-fp8 path (BASELINE.json configs[4] "fp8 MFMA weight path") on the GPU vs oracle/mx_ref.py.

* quantizer (f32 rows -> e4m3 + E8M0): bit-exact;
* LayerNorm with MX output: codes / scales of the oracle's quantization of the f64 LN, up to
  rounding-boundary flips (the LN itself runs in f32);
* MX GEMM on oracle-quantized operands: f32 epilogues within 2^-12 of sum |a||w| (the
  block-scaled MFMA does not accumulate its 64 products exactly in f32: measured
  (tools/mx_diag.py) max error ~2^-15 of sum |a||w| on random data, exact on small
  integers); 16-bit epilogue within one 16-bit ulp; the quantizing epilogue (c_fc -> c_proj)
  against the oracle's quantization of the f64 result.
"""
import numpy as np
import pytest

from oracle import clip_ref, mx_ref

pytestmark = pytest.mark.gpu

BF16 = 0


def _lib():
    from open_clip_inference import _lib
    return _lib


def ref_act(act, x):
    return {0: lambda v: v, 1: lambda v: clip_ref.act_fn("quick_gelu", v),
            2: lambda v: clip_ref.act_fn("gelu", v), 3: lambda v: clip_ref.act_fn("gelu_tanh", v)}[act](x)


def _rows(rng, R, C, spread=True):
    x = rng.standard_normal((R, C)).astype(np.float32)
    if spread:  # per-block magnitudes over many binades, zeros, a denormal block
        x *= np.exp2(rng.integers(-12, 12, size=(R, C // 32, 1))).repeat(32, -1).reshape(R, C).astype(np.float32)
        x[0, :32] = 0.0
        if R > 1:
            x[1, :32] = np.float32(1e-40)
    return x


@pytest.mark.parametrize("R,C", [(1, 32), (37, 96), (513, 1280), (64, 4096)])
def test_quant_rows_bit_exact(R, C):
    L = _lib()
    x = _rows(np.random.default_rng(R + C), R, C)
    q = np.empty((R, C), np.uint8)
    s = np.empty((R, C // 32), np.uint8)
    L.check(L.lib().clipgpu_test_quant_rows(R, C, x.ctypes.data, q.ctypes.data, s.ctypes.data))
    rq, rs = mx_ref.quantize_rows(x)
    np.testing.assert_array_equal(s, rs)
    np.testing.assert_array_equal(q, rq)


@pytest.mark.parametrize("D", [128, 768, 1024, 1280])
def test_layernorm_mx(D):
    L = _lib()
    rng = np.random.default_rng(D)
    rows = 257
    x = (rng.standard_normal((rows, D)) * 3 + 1).astype(np.float32)
    w = (1 + 0.3 * rng.standard_normal(D)).astype(np.float32)
    b = (0.1 * rng.standard_normal(D)).astype(np.float32)
    q = np.empty((rows, D), np.uint8)
    s = np.empty((rows, D // 32), np.uint8)
    L.check(L.lib().clipgpu_test_layernorm_mx(rows, D, 1e-5, x.ctypes.data, w.ctypes.data, b.ctypes.data,
                                              q.ctypes.data, s.ctypes.data))
    ref = clip_ref.layer_norm(x.astype(np.float64), w, b, 1e-5)
    rq, rs = mx_ref.quantize_rows(ref.astype(np.float32))
    # f32 LN vs f64: a value within ~1e-6 of a rounding midpoint / a block amax at a scale
    # boundary may land on the neighbouring code
    assert (s == rs).mean() > 0.999
    assert (q == rq).mean() > 0.995
    deq = mx_ref.dequantize(q, s)
    # half the e4m3 spacing at the top binade of the block ([256, 448] * 2^e: spacing 2^(e+5))
    half = np.ldexp(1.0, s.astype(np.int64) - 127 + 4).repeat(32, -1)
    assert np.all(np.abs(deq - ref) <= half * 1.01)


def _mx_operands(rng, M, N, K):
    A = rng.standard_normal((M, K)).astype(np.float32)
    W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
    aq, as_ = mx_ref.quantize_rows(A)
    wq, ws = mx_ref.quantize_rows(W)
    return aq, as_, wq, ws


def run_gemm_mx(mode, act, aq, as_, wq, ws, bias=None, resid=None):
    L = _lib()
    M, K = aq.shape
    N = wq.shape[0]
    out = np.empty((M, N), np.float32)
    outq = np.empty((M, N), np.uint8)
    outs = np.empty((M, N // 32), np.uint8)
    b = None if bias is None else np.ascontiguousarray(bias, np.float32)
    r = None if resid is None else np.ascontiguousarray(resid, np.float32)
    L.check(L.lib().clipgpu_test_gemm_mx(BF16, mode, act, M, N, K, aq.ctypes.data, as_.ctypes.data, wq.ctypes.data,
                                         ws.ctypes.data, None if b is None else b.ctypes.data,
                                         None if r is None else r.ctypes.data, out.ctypes.data, outq.ctypes.data,
                                         outs.ctypes.data))
    return out, outq, outs


@pytest.fixture(params=[0, 2, 3], ids=["auto", "mx256x128", "mx128x128"])
def mx_tile(request, monkeypatch):
    monkeypatch.setenv("CLIPGPU_TEST_TILE", str(request.param))
    return request.param


@pytest.mark.parametrize("M,N,K", [(128, 128, 128), (200, 160, 256), (1000, 768, 768), (77, 64, 512),
                                   (3000, 1280, 1280), (2053, 384, 640)])
def test_gemm_mx_f32(M, N, K, mx_tile):
    rng = np.random.default_rng(M + N + K)
    aq, as_, wq, ws = _mx_operands(rng, M, N, K)
    bias = rng.standard_normal(N).astype(np.float32)
    out, _, _ = run_gemm_mx(2, 0, aq, as_, wq, ws, bias)
    ref = mx_ref.mx_gemm_ref(aq, as_, wq, ws, bias)
    bound = np.abs(mx_ref.dequantize(aq, as_)) @ np.abs(mx_ref.dequantize(wq, ws)).T + np.abs(bias)
    assert np.all(np.abs(out - ref) <= 2.0 ** -12 * bound + 1e-30)


def test_gemm_mx_residual(mx_tile):
    rng = np.random.default_rng(5)
    M, N, K = 700, 512, 1024
    aq, as_, wq, ws = _mx_operands(rng, M, N, K)
    bias = rng.standard_normal(N).astype(np.float32)
    resid = rng.standard_normal((M, N)).astype(np.float32)
    out, _, _ = run_gemm_mx(1, 0, aq, as_, wq, ws, bias, resid)
    ref = mx_ref.mx_gemm_ref(aq, as_, wq, ws, bias) + resid
    bound = np.abs(mx_ref.dequantize(aq, as_)) @ np.abs(mx_ref.dequantize(wq, ws)).T + np.abs(bias) + np.abs(resid)
    assert np.all(np.abs(out - ref) <= 2.0 ** -12 * bound)


@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_gemm_mx_store16_act(act, mx_tile):
    rng = np.random.default_rng(10 + act)
    M, N, K = 600, 384, 768
    aq, as_, wq, ws = _mx_operands(rng, M, N, K)
    bias = rng.standard_normal(N).astype(np.float32)
    out, _, _ = run_gemm_mx(0, act, aq, as_, wq, ws, bias)
    ref = ref_act(act, mx_ref.mx_gemm_ref(aq, as_, wq, ws, bias))
    # bf16 output rounding (2^-9 relative) + MFMA accumulation + fast activation forms
    bound = np.abs(mx_ref.dequantize(aq, as_)) @ np.abs(mx_ref.dequantize(wq, ws)).T + np.abs(bias)
    assert np.all(np.abs(out - ref) <= 2.0 ** -8 * np.abs(ref) + 2.0 ** -12 * bound)


@pytest.mark.parametrize("act", [0, 2])
def test_gemm_mx_quantized_out(act, mx_tile):
    rng = np.random.default_rng(20 + act)
    M, N, K = 900, 1280, 640
    aq, as_, wq, ws = _mx_operands(rng, M, N, K)
    bias = rng.standard_normal(N).astype(np.float32)
    _, q, s = run_gemm_mx(3, act, aq, as_, wq, ws, bias)
    ref = ref_act(act, mx_ref.mx_gemm_ref(aq, as_, wq, ws, bias))
    rq, rs = mx_ref.quantize_rows(ref.astype(np.float32))
    assert (s == rs).mean() > 0.999
    assert (q == rq).mean() > 0.995
    deq = mx_ref.dequantize(q, s)
    half = np.ldexp(1.0, s.astype(np.int64) - 127 + 4).repeat(32, -1)
    assert np.all(np.abs(deq - ref) <= half * 1.01)


def test_gemm_mx_rejects_bad_shapes():
    L = _lib()
    rng = np.random.default_rng(0)
    aq, as_, wq, ws = _mx_operands(rng, 64, 64, 128)
    with pytest.raises(L.ClipError):
        run_gemm_mx(2, 0, aq[:, :96].copy(), as_[:, :3].copy(), wq[:, :96].copy(), ws[:, :3].copy())


# ---- fp8 engines end to end ------------------------------------------------------------------
# The fp8 path is lossy by construction (e4m3 keeps 3 mantissa bits), and the reference has no
# fp8 arithmetic to match bit-wise.  The per-site ablation (tools/mx_ablation.py, DESIGN.md §1,
# profiles/r02_mx_ablation.jsonl) shows every MX site costs cosine roughly additively and that no
# split with a useful speed-up keeps the bf16 path's 0.9999: the default split (QKV, c_fc, c_proj)
# measured min 0.99920-0.99944 on the vision towers and 0.99442-0.99491 on the text towers against
# the fp32 reference.  These are the bars the shipped split meets (against the fp64 oracle on the
# seeded weights); the QKV-only split meets the north-star bar on the CLIP vision towers.
FP8_COS_VISION = 0.999
FP8_COS_TEXT = 0.993
FP8_COS = FP8_COS_VISION


def _fp8_check(got, ref, label, bar=None):
    bar = (FP8_COS_TEXT if "text" in label else FP8_COS_VISION) if bar is None else bar
    cos = clip_ref.cosine_rows(got, ref)
    print(f"\n[fp8] {label}: cos min {cos.min():.6f} mean {cos.mean():.6f}")
    assert np.all(np.abs(np.linalg.norm(got, axis=1) - 1) < 1e-5)
    assert cos.min() >= bar, cos.min()
    return cos


def _engine(cfg, tower, dtype, max_batch, **opts):
    from open_clip_inference.engine import Engine
    from tests.helpers import make_model_dir
    return Engine(make_model_dir(cfg, 1234), tower, [0], dtype, max_batch, **opts)


def test_fp8_vit_b32_vision_and_text():
    from oracle import weights
    from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, VIT_B_32_CFG
    from tests.helpers import normalized_pixels, specs
    v, t = specs(VIT_B_32_CFG)
    u8 = weights.synth_images_u8(5, 6, v.image_size)
    px = normalized_pixels(u8, OPENAI_MEAN, OPENAI_STD)
    e = _engine(VIT_B_32_CFG, 0, "fp8", 16)
    got = e.embed_pixels(px)
    _fp8_check(got, clip_ref.encode_image(weights.vision_weights(v, 1234), v, px), "ViT-B/32 vision")
    assert np.array_equal(got, e.embed_pixels(px))  # deterministic
    ids = weights.synth_token_ids(6, 5, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                  random_eot=True)
    te = _engine(VIT_B_32_CFG, 1, "fp8", 16)
    _fp8_check(te.embed_tokens(ids), clip_ref.encode_text(weights.text_weights(t, 1234), t, ids), "ViT-B/32 text")


def test_fp8_lanes_and_batch_split_are_bit_exact():
    """Row results do not depend on the batch composition or the lane split (no cross-row state
    in the MX quantization: scales are per row)."""
    from oracle import weights
    from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, VIT_B_32_CFG
    from tests.helpers import normalized_pixels, specs
    v, _ = specs(VIT_B_32_CFG)
    px = normalized_pixels(weights.synth_images_u8(8, 40, v.image_size), OPENAI_MEAN, OPENAI_STD)
    heur = [-1, -1, -1, -1]
    a = _engine(VIT_B_32_CFG, 0, "fp8", 64, gemm_tiles=heur, lanes=2).embed_pixels(px)
    b = _engine(VIT_B_32_CFG, 0, "fp8", 64, gemm_tiles=heur, lanes=1).embed_pixels(px)
    assert np.array_equal(a, b)


def test_fp8_vit_h14_378_full_dims():
    """BASELINE configs[4] (DFN5B ViT-H/14-378 vision + text, fp8 MFMA weight path) at full dims."""
    from oracle import weights
    from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, VIT_H_14_378_CFG
    from tests.helpers import normalized_pixels, specs
    v, t = specs(VIT_H_14_378_CFG)
    px = normalized_pixels(weights.synth_images_u8(3, 2, v.image_size), OPENAI_MEAN, OPENAI_STD)
    e = _engine(VIT_H_14_378_CFG, 0, "fp8", 2)
    _fp8_check(e.embed_pixels(px), clip_ref.encode_image(weights.vision_weights(v, 1234), v, px), "ViT-H/14-378 vision")
    ids = weights.synth_token_ids(4, 3, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                  random_eot=True)
    te = _engine(VIT_H_14_378_CFG, 1, "fp8", 3)
    _fp8_check(te.embed_tokens(ids), clip_ref.encode_text(weights.text_weights(t, 1234), t, ids), "ViT-H/14 text")


def test_fp8_so400m_siglip2_full_dims():
    from oracle import weights
    from oracle.model_spec import SIGLIP_MEAN, SIGLIP_STD, SO400M_16_SIGLIP2_384_CFG
    from tests.helpers import normalized_pixels, specs
    v, _ = specs(SO400M_16_SIGLIP2_384_CFG)
    px = normalized_pixels(weights.synth_images_u8(7, 2, v.image_size), SIGLIP_MEAN, SIGLIP_STD)
    e = _engine(SO400M_16_SIGLIP2_384_CFG, 0, "fp8", 2)
    _fp8_check(e.embed_pixels(px), clip_ref.encode_image(weights.vision_weights(v, 1234), v, px), "SO400M vision")


def test_fp8_tiny_and_rejects_unsupported_width():
    import copy
    from open_clip_inference import _lib as L
    from oracle import weights
    from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, TINY_CFG
    from tests.helpers import normalized_pixels, specs
    v, _ = specs(TINY_CFG)
    px = normalized_pixels(weights.synth_images_u8(9, 3, v.image_size), OPENAI_MEAN, OPENAI_STD)
    got = _engine(TINY_CFG, 0, "fp8", 4).embed_pixels(px)
    _fp8_check(got, clip_ref.encode_image(weights.vision_weights(v, 1234), v, px), "tiny vision")
    cfg = copy.deepcopy(TINY_CFG)
    cfg["model_cfg"]["vision_cfg"]["width"] = 192  # 3 heads of 64: not a multiple of 128
    with pytest.raises(L.ClipError):
        _engine(cfg, 0, "fp8", 4)


def test_fp8_input_paths_agree():
    """fp8 engines share the bf16 engines' stems: u8 input (normalised while staging the patch
    rows) gives the f32 path's embeddings bit for bit, and the device-side photo resize path
    (clipgpu_embed_images_rgb8) equals host preprocess + embed_pixels; a two-replica handle
    shards in input order."""
    from oracle import weights
    from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, VIT_B_32_CFG
    from tests.helpers import normalized_pixels, specs
    from open_clip_inference.engine import Engine, preprocess_batch_rgb8
    from tests.helpers import make_model_dir
    v, _ = specs(VIT_B_32_CFG)
    u8 = weights.synth_images_u8(12, 5, v.image_size)
    e = _engine(VIT_B_32_CFG, 0, "fp8", 8)
    assert np.array_equal(e.embed_u8(u8, OPENAI_MEAN, OPENAI_STD),
                          e.embed_pixels(normalized_pixels(u8, OPENAI_MEAN, OPENAI_STD)))
    rng = np.random.default_rng(3)
    ims = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in ((480, 640), (300, 200), (224, 224))]
    host = e.embed_pixels(preprocess_batch_rgb8(ims, 224, "bicubic", "shortest", OPENAI_MEAN, OPENAI_STD))
    assert np.array_equal(e.embed_images_rgb8(ims), host)
    multi = Engine(make_model_dir(VIT_B_32_CFG, 1234), 0, [0, 0], "fp8", 2)
    assert np.array_equal(multi.embed_images_rgb8(ims), host)


@pytest.mark.parametrize("cfg_name", ["VIT_B_32_CFG", "VIT_H_14_378_CFG"])
def test_fp8_qkv_only_split_meets_the_north_star_bar_on_clip_vision(cfg_name):
    """mx_sites = qkv (only the QKV projection in MX-fp8): the CLIP vision towers keep
    cos >= 0.9999 against the fp64 oracle (the ablation's one split that does)."""
    from oracle import model_spec, weights
    from oracle.model_spec import OPENAI_MEAN, OPENAI_STD
    from tests.helpers import COS_TOL, normalized_pixels, specs
    cfg = getattr(model_spec, cfg_name)
    v, _ = specs(cfg)
    px = normalized_pixels(weights.synth_images_u8(13, 2, v.image_size), OPENAI_MEAN, OPENAI_STD)
    e = _engine(cfg, 0, "fp8", 2, mx_sites="qkv")
    _fp8_check(e.embed_pixels(px), clip_ref.encode_image(weights.vision_weights(v, 1234), v, px),
               f"{cfg_name} vision, MX at QKV only", bar=COS_TOL)


def test_fp8_site_selection_is_validated():
    from open_clip_inference import _lib as L
    from oracle.model_spec import VIT_B_32_CFG
    with pytest.raises(L.ClipError, match="proj in MX needs fc"):
        _engine(VIT_B_32_CFG, 0, "fp8", 2, mx_sites="proj")
    with pytest.raises(L.ClipError, match="mx_layers needs dtype"):
        _engine(VIT_B_32_CFG, 0, "bf16", 2, mx_layers=[0])
