"""Clip facade (open_clip_inference.clip, mirror of src/clip.rs) vs oracle/facade_ref.py.
Embedders are replaced by fixed-embedding fakes so this runs without a GPU; the GPU
end-to-end version is tests/test_gpu_api.py."""
import numpy as np
import pytest

from oracle import facade_ref
from open_clip_inference.clip import Clip
from open_clip_inference.config import ModelConfig


class FakeVision:
    def __init__(self, embs):
        self.embs = embs

    def embed_image(self, img):
        return self.embs[img]

    def embed_images(self, imgs):
        return np.stack([self.embs[i] for i in imgs])


class FakeText:
    def __init__(self, embs, mc):
        self.embs = embs
        self.model_config = mc

    def embed_text(self, t):
        return self.embs[t]

    def embed_texts(self, ts):
        return np.stack([self.embs[t] for t in ts])


def unit(rng, n, d=32):
    x = rng.standard_normal((n, d)).astype(np.float32)
    return x / np.linalg.norm(x, axis=1, keepdims=True)


@pytest.mark.parametrize("mc", [ModelConfig(logit_scale=100.0, logit_bias=0.0, activation_function="softmax"),
                                ModelConfig(logit_scale=10.0, logit_bias=-10.0, activation_function="sigmoid"),
                                ModelConfig()])
def test_classify_rank_compare(mc):
    rng = np.random.default_rng(1)
    ie = unit(rng, 4)
    te = unit(rng, 3)
    labels = ["A photo of a cat", "A photo of a dog", "A photo of a beignet"]
    clip = Clip(FakeVision({i: ie[i] for i in range(4)}), FakeText(dict(zip(labels, te)), mc), "/x")
    scale = 1.0 if mc.logit_scale is None else mc.logit_scale
    bias = 0.0 if mc.logit_bias is None else mc.logit_bias
    act = mc.activation_function or "softmax"
    got = clip.classify(0, labels)
    ref = facade_ref.classify(ie[0], te, labels, scale, bias, act)
    assert [l for l, _ in got] == [l for l, _ in ref]
    assert np.allclose([p for _, p in got], [p for _, p in ref], rtol=1e-5, atol=1e-7)
    got = clip.rank_images([0, 1, 2, 3], labels[1])
    ref = facade_ref.rank_images(ie, te[1], scale, bias, act)
    assert [i for i, _ in got] == [i for i, _ in ref]
    assert np.allclose([p for _, p in got], [p for _, p in ref], rtol=1e-5, atol=1e-7)
    assert abs(clip.compare(2, labels[2]) - facade_ref.compare(ie[2], te[2], scale, bias)) < 1e-4


def test_softmax_sigmoid_static():
    x = [1.0, 2.0, 3.0, -1000.0]
    assert np.allclose(Clip.softmax(x), facade_ref.softmax(x), rtol=1e-6)
    assert abs(sum(Clip.softmax(x)) - 1) < 1e-6
    assert abs(Clip.sigmoid(0.0) - 0.5) < 1e-7
    assert abs(Clip.sigmoid(3.0) - facade_ref.sigmoid(3.0)) < 1e-7


@pytest.mark.parametrize("mc", [ModelConfig(logit_scale=100.0, logit_bias=0.0, activation_function="softmax"),
                                ModelConfig(logit_scale=117.33, logit_bias=-12.9, activation_function="sigmoid"),
                                ModelConfig(logit_scale=100.0, logit_bias=-16.5, activation_function="softmax"),
                                ModelConfig()])
@pytest.mark.parametrize("E,n", [(512, 3), (768, 17), (1152, 64), (37, 5)])
def test_facade_is_bit_exact_to_the_reference_f32_arithmetic(mc, E, n):
    """compare / classify / rank_images give the reference's f32 bits (src/clip.rs:79-185):
    ndarray's eight-accumulator unrolled dot, one fused mul_add (logit_bias != 0 included), libm
    expf, a sequential f32 softmax sum -- against the exact restatement in oracle/facade_ref.py
    (rational fused multiply-add).  E = 37 covers the unrolled dot's < 8-element tail."""
    rng = np.random.default_rng(E + n)
    ie = unit(rng, n, E)
    te = unit(rng, n, E)
    labels = [f"label {i}" for i in range(n)]
    clip = Clip(FakeVision({i: ie[i] for i in range(n)}), FakeText(dict(zip(labels, te)), mc), "/x")
    scale = np.float32(1.0 if mc.logit_scale is None else mc.logit_scale)
    bias = np.float32(0.0 if mc.logit_bias is None else mc.logit_bias)
    act = mc.activation_function or "softmax"
    got = clip.classify(0, labels)
    ref = facade_ref.classify_f32_exact(ie[0], te, labels, scale, bias, act)
    assert got == ref
    got = clip.rank_images(list(range(n)), labels[1])
    ref = facade_ref.rank_images_f32_exact(ie, te[1], scale, bias, act)
    assert got == ref
    for i in range(min(n, 4)):
        c = clip.compare(i, labels[i])
        r = facade_ref.scores_f32_exact(ie[i][None], te[i], scale, bias, "logits")[0]
        assert np.float32(c).tobytes() == np.float32(r).tobytes()


def test_facade_mul_add_is_fused():
    """A case where one rounding (mul_add) and two roundings (multiply, then add) differ: the
    facade must give the fused result (src/clip.rs:89)."""
    a, b, c = np.float32(1 + 2 ** -12), np.float32(1.0), np.float32(-(1 + 2 ** -11))
    # sim = a . a = 1 + 2^-11 + 2^-24 rounds (tie to even) to 1 + 2^-11 in f32; the logit is
    # sim.mul_add(b, c): with the rounded sim both forms give 0, so feed the product through the
    # scale instead: logit = a.mul_add(a, c) = 2^-24 exactly, a * a + c = 0
    fused = facade_ref.mul_add_f32(a, a, c)
    assert fused == np.float32(2.0 ** -24)
    assert np.float32(np.float32(a * a) + c) == np.float32(0)
    clip = Clip(FakeVision({0: np.array([b], np.float32)}),
                FakeText({"t": np.array([a], np.float32)}, ModelConfig(logit_scale=float(a), logit_bias=float(c))),
                "/x")
    assert np.float32(clip.compare(0, "t")) == fused


def test_softmax_sigmoid_statics_match_reference():
    x = np.array([3.5, -1.25, 100.0, 99.9, 0.0], np.float32)
    assert [np.float32(v) for v in Clip.softmax(x)] == facade_ref.softmax_f32(x)
    for l in (-30.0, -0.5, 0.0, 2.25, 40.0):
        assert np.float32(Clip.sigmoid(l)) == facade_ref.sigmoid_f32(l)
