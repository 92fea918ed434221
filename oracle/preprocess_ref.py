"""numpy restatement of VisionEmbedder preprocessing — TEST INFRASTRUCTURE.

src/vision.rs:119-259: crop box (f64) of resize_with_fast_image_resize (:184-192),
separable convolution resize (CatmullRom for "bicubic", triangle for "bilinear",
:176-180), normalize_pixels (:235-259).  The convolution restates the scheme
fast_image_resize 6.0.0 shares with Pillow's Resample.c (filter support scaled by
the downscale factor, normalised coefficients, fixed point, horizontal pass then
vertical pass through a u8 intermediate) with Pillow's 22-bit rounding; pinned
against Pillow 12.2 (tests/test_cpu_preprocess.py).  Small images only (Python loops).
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _cubic(x, a=-0.5):
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def _triangle(x):
    x = abs(x)
    return 1.0 - x if x < 1.0 else 0.0


def crop_box(W, H, S, mode="shortest"):
    if mode == "squash":
        return 0.0, 0.0, float(W), float(H)
    scale = S / min(W, H)
    cw = S / scale
    x0, y0 = (W - cw) / 2.0, (H - cw) / 2.0
    return max(0.0, x0), max(0.0, y0), min(float(W), x0 + cw), min(float(H), y0 + cw)


def _coeffs(in_size, in0, in1, out_size, filt, support0):
    scale = (in1 - in0) / out_size
    fs = max(scale, 1.0)
    support = support0 * fs
    out = []
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [filt((x + xmin - center + 0.5) / fs) for x in range(xmax)]
        ww = sum(w)
        w = [v / ww if ww != 0.0 else v for v in w]
        k = [int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS)) for v in w]
        out.append((xmin, np.array(k, np.int64)))
    return out


def _clip8(v):
    v = v >> PRECISION_BITS
    return np.clip(v, 0, 255).astype(np.uint8)


def resize(rgb: np.ndarray, S: int, interpolation="bicubic", mode="shortest") -> np.ndarray:
    H, W = rgb.shape[:2]
    x0, y0, x1, y1 = crop_box(W, H, S, mode)
    filt, sup = (_cubic, 2.0) if interpolation == "bicubic" else (_triangle, 1.0)
    ch = _coeffs(W, x0, x1, S, filt, sup)
    cv = _coeffs(H, y0, y1, S, filt, sup)
    need_h = S != W or x0 != 0.0 or x1 != S
    need_v = S != H or y0 != 0.0 or y1 != S
    src = rgb.astype(np.int64)
    if need_h:
        yfirst = cv[0][0]
        ylast = cv[-1][0] + len(cv[-1][1])
        rows = src[yfirst:ylast]
        tmp = np.empty((ylast - yfirst, S, 3), np.uint8)
        for xx, (xmin, k) in enumerate(ch):
            acc = (rows[:, xmin:xmin + len(k)] * k[None, :, None]).sum(1) + (1 << (PRECISION_BITS - 1))
            tmp[:, xx] = _clip8(acc)
        src = tmp.astype(np.int64)
        cv = [(ymin - yfirst, k) for ymin, k in cv]
    if not need_v:
        return src[:S].astype(np.uint8)
    out = np.empty((S, S, 3), np.uint8)
    for yy, (ymin, k) in enumerate(cv):
        acc = (src[ymin:ymin + len(k)] * k[:, None, None]).sum(0) + (1 << (PRECISION_BITS - 1))
        out[yy] = _clip8(acc)
    return out


def normalize_pixels(rgb: np.ndarray, mean, std) -> np.ndarray:
    """[S,S,3] u8 -> [3,S,S] f32: (p / 255 - mean[c]) / std[c] in f32 (src/vision.rs:251-256)."""
    x = rgb.astype(np.float32) / np.float32(255.0)
    x = (x - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return np.ascontiguousarray(x.transpose(2, 0, 1))


def preprocess(rgb, S, mean, std, interpolation="bicubic", mode="shortest"):
    return normalize_pixels(resize(rgb, S, interpolation, mode), mean, std)
