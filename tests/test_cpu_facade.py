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
