"""Host preprocessing (csrc/host/preprocess.cpp, the product) vs the oracle restatement
(oracle/preprocess_ref.py, bit-exact) and vs Pillow 12.2 (the independent pin of the
convolution scheme: within 1 u8 level).  The product follows fast_image_resize 6.0.0's u8
convolution (a5, the reference's default feature): i16 coefficients at the adaptive precision
of its Normalizer16, where Pillow 12.2 keeps 22-bit coefficients -- the two differ by at most one
level on under 1 % of samples.  normalize_pixels is bit-exact (f32 divide as
src/vision.rs:254-255)."""
import os

import numpy as np
import pytest

from oracle import preprocess_ref
from oracle.model_spec import OPENAI_MEAN, OPENAI_STD
from oracle.weights import synth_images_u8

GOLD = os.path.join(os.path.dirname(__file__), "golden", "preprocess_golden.npz")


def cpp_resize(rgb, S, interp="bicubic", mode="shortest"):
    from open_clip_inference.engine import resize_rgb8
    return resize_rgb8(rgb, S, interp, mode)


def cpp_preprocess(images, S, interp="bicubic", mode="shortest", mean=OPENAI_MEAN, std=OPENAI_STD):
    from open_clip_inference.engine import preprocess_batch_rgb8
    return preprocess_batch_rgb8(images, S, interp, mode, mean, std)


def synth(h, w):
    return synth_images_u8(h * 1000 + w, 1, max(h, w))[0][:h, :w].copy()


def close_to(a, b, exact_frac=0.99):
    d = np.abs(a.astype(np.int32) - b.astype(np.int32))
    assert d.max() <= 1, d.max()
    assert (d == 0).mean() >= exact_frac, (d == 0).mean()


@pytest.mark.parametrize("hw", [(389, 517), (300, 200), (64, 64), (97, 301), (50, 40)])
@pytest.mark.parametrize("mode", ["shortest", "squash"])
def test_resize_vs_pillow_golden(hw, mode):
    g = np.load(GOLD)
    h, w = hw
    key = f"synth_{h}x{w}_64" + ("_squash" if mode == "squash" else "")
    close_to(cpp_resize(synth(h, w), 64, "bicubic", mode), g[key])


def test_resize_real_photo_vs_pillow():
    g = np.load(GOLD)
    crop = g["cat_face_crop"]
    close_to(cpp_resize(crop, 224), g["cat_face_crop_224"])
    close_to(cpp_resize(crop, 64, "bilinear"), g["cat_face_crop_64_bilinear"])


@pytest.mark.parametrize("hw,S,interp,mode", [((389, 517), 64, "bicubic", "shortest"),
                                             ((120, 77), 224, "bicubic", "shortest"),
                                             ((97, 301), 48, "bilinear", "squash"),
                                             ((64, 64), 64, "bicubic", "shortest"),
                                             ((200, 64), 64, "bicubic", "shortest")])
def test_resize_bit_exact_vs_oracle(hw, S, interp, mode):
    img = synth(*hw)
    assert np.array_equal(cpp_resize(img, S, interp, mode), preprocess_ref.resize(img, S, interp, mode))


def test_identity_resize_for_presized_input():
    """Synthetic S x S inputs: crop is the full image and the resize is the identity."""
    img = synth(224, 224)
    assert np.array_equal(cpp_resize(img, 224), img)


def test_normalize_bit_exact_and_batch_layout():
    imgs = [synth(300, 200), synth(64, 64), synth(97, 301)]
    out = cpp_preprocess(imgs, 64)
    assert out.shape == (3, 3, 64, 64) and out.dtype == np.float32
    for i, im in enumerate(imgs):
        ref = preprocess_ref.preprocess(im, 64, OPENAI_MEAN, OPENAI_STD)
        assert np.array_equal(out[i], ref)


def test_empty_batch_error():
    from open_clip_inference.error import InferenceError
    with pytest.raises(InferenceError, match="Empty batch"):
        cpp_preprocess([], 64)


def test_nearest_mode_runs():
    out = cpp_resize(synth(100, 150), 32, "nearest")
    assert out.shape == (32, 32, 3)


IMAGE_CRATE_SIZES = [(389, 517), (97, 301), (224, 224), (600, 450), (64, 64), (33, 70), (1, 400), (700, 1),
                     (500, 500), (81, 64), (225, 223), (122, 162)]


@pytest.mark.parametrize("interp", ["bicubic", "bilinear", "nearest"])
@pytest.mark.parametrize("mode", ["shortest", "squash"])
@pytest.mark.parametrize("S", [224, 64])
def test_resize_with_image_bit_exact_vs_restatement(interp, mode, S):
    """a6, resize_with_image (src/vision.rs:200-233; the crate without `fast_image_resize`): the
    C++ path equals the f32 restatement of image 0.25.9's imageops::resize + crop_imm bit for bit
    (oracle/preprocess_ref.py) -- down- and up-scaling, identity sizes, 1-pixel-wide images, the
    decoded cat_face crop."""
    from open_clip_inference.engine import resize_rgb8
    rng = np.random.default_rng(S + len(interp) + len(mode))
    g = np.load(GOLD)
    ims = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in IMAGE_CRATE_SIZES] + [g["cat_face_crop"]]
    for im in ims:
        ref = preprocess_ref.resize_with_image(im, S, interp, mode)
        got = resize_rgb8(im, S, interp, mode, resize_impl="image")
        assert got.shape == (S, S, 3)
        assert np.array_equal(got, ref), (im.shape, int(np.abs(got.astype(int) - ref).max()))


@pytest.mark.parametrize("interp,pil", [("bicubic", "BICUBIC"), ("bilinear", "BILINEAR"), ("nearest", "NEAREST")])
def test_resize_with_image_near_pillow_when_downscaling(interp, pil):
    """Anchor for the restatement (the image crate itself is not in this image): Pillow's
    resize of the whole image to round(W*s) x round(H*s) then the same crop -- the same filters
    (CatmullRom = Keys a=-0.5, triangle, nearest) in fixed point -- agrees within one level when
    downscaling.  Parity with the crate itself is unpinned."""
    from PIL import Image
    rng = np.random.default_rng(7)
    for h, w in [(389, 517), (97, 301), (600, 450), (500, 500)]:
        im = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        im = (np.cumsum(im.astype(np.int64), axis=1) // np.arange(1, w + 1)[None, :, None]).astype(np.uint8)
        S = 64
        a = preprocess_ref.resize_with_image(im, S, interp, "shortest")
        scale = np.float32(S) / np.float32(min(w, h))
        sw, sh = int(np.floor(np.float32(w * scale) + 0.5)), int(np.floor(np.float32(h * scale) + 0.5))
        r = np.asarray(Image.fromarray(im).resize((sw, sh), getattr(Image, pil)))
        x, y = int(np.floor((sw - S) / 2 + 0.5)), int(np.floor((sh - S) / 2 + 0.5))
        assert np.abs(a.astype(int) - r[y:y + S, x:x + S]).max() <= 1


def test_preprocess_batch_image_backend():
    """preprocess_batch with the image-crate resize (clipgpu_preprocess_batch_image, thread pool)
    = normalize_pixels of the restated resize, bit for bit; empty batch is an error."""
    from open_clip_inference.engine import preprocess_batch_rgb8
    from open_clip_inference.error import InferenceError
    rng = np.random.default_rng(3)
    ims = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in [(389, 517), (97, 301), (64, 64)]]
    got = preprocess_batch_rgb8(ims, 64, "bicubic", "shortest", OPENAI_MEAN, OPENAI_STD, resize_impl="image")
    for i, im in enumerate(ims):
        px = preprocess_ref.resize_with_image(im, 64, "bicubic", "shortest")
        ref = preprocess_ref.normalize_pixels(px, OPENAI_MEAN, OPENAI_STD)
        assert np.array_equal(got[i], ref)
    with pytest.raises(InferenceError, match="Empty batch"):
        preprocess_batch_rgb8([], 64, "bicubic", "shortest", OPENAI_MEAN, OPENAI_STD, resize_impl="image")


@pytest.mark.parametrize("in_size,out_size,filt", [(517, 64, "bicubic"), (389, 224, "bicubic"), (120, 224, "bicubic"),
                                                   (224, 224, "bicubic"), (97, 48, "bilinear"), (50, 400, "bilinear")])
def test_fast_image_resize_coefficient_precision(in_size, out_size, filt):
    """Normalizer16 (fast_image_resize 6.0.0, ported from Pillow-SIMD): the axis precision p is the
    largest p < 22 with round(max weight * 2^p) < 2^15 (i16 headroom; round(max w * 2^(p+1)) no longer fits), every
    coefficient is round-half-away(w * 2^p) and fits an i16, and each output's coefficients sum to
    2^p within the rounding of its taps."""
    f, sup = (preprocess_ref._cubic, 2.0) if filt == "bicubic" else (preprocess_ref._triangle, 1.0)
    rows, p = preprocess_ref._coeffs(in_size, 0.0, float(in_size), out_size, f, sup)
    wmax = 0.0
    for _, k in rows:
        wmax = max(wmax, float(k.max()) / (1 << p))
    assert 4 <= p < 22
    assert round(wmax * (1 << (p + 1))) >= (1 << 15) or p == 21
    assert round(wmax * (1 << p)) < (1 << 15)
    for _, k in rows:
        assert np.all(np.abs(k) < 32768)
        assert abs(int(k.sum()) - (1 << p)) <= len(k)
    if in_size == out_size:  # identity: one unit tap per output, exact copy
        assert p == 14 and all(int(k.max()) == 1 << 14 for _, k in rows)
