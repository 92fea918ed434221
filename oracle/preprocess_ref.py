"""numpy restatement of VisionEmbedder preprocessing — TEST INFRASTRUCTURE.

src/vision.rs:119-259: crop box (f64) of resize_with_fast_image_resize (:184-192),
separable convolution resize (CatmullRom for "bicubic", triangle for "bilinear",
:176-180), normalize_pixels (:235-259).  The convolution restates fast_image_resize
6.0.0's u8 path (the crate is not installable here; restated from its published
algorithm, a port of Pillow-SIMD): precompute_coefficients (taps floor(c - r) ..
ceil(c + r), weights filter((x - (c - 0.5)) / max(scale, 1)) normalised by their sum)
then Normalizer16 (i16 coefficients at the largest precision p < 22 with
round(max weight * 2^p) < 2^15, so p = 14 for a unit tap; rounded half away from zero), i32 sums from
2^(p-1), clamp(sum >> p, 0, 255), horizontal pass then vertical pass through a u8
intermediate.  Pinned against Pillow 12.2 within one level (its 22-bit scheme;
tests/test_cpu_preprocess.py).  Small images only (Python loops).
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2  # fast_image_resize / Pillow-SIMD: the precision search's bound
MAX_COEFS_PRECISION = 16 - 1  # i16 coefficients


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
    """[(first tap, i16 coefficients)] per output and the axis precision p (see header)."""
    scale = (in1 - in0) / out_size
    fs = max(scale, 1.0)
    radius = support0 * fs
    recip = 1.0 / fs
    rows = []
    for xx in range(out_size):
        in_center = in0 + (xx + 0.5) * scale
        xmin = int(max(math.floor(in_center - radius), 0.0))
        xmax = min(int(math.ceil(in_center + radius)), in_size)
        center = in_center - 0.5
        w = [filt((x - center) * recip) for x in range(xmin, xmax)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        rows.append((xmin, w))
    wmax = max(max(w) if w else 0.0 for _, w in rows)
    if any(len(w) < int(math.ceil(radius)) * 2 + 1 for _, w in rows):
        wmax = max(wmax, 0.0)  # the zero padding of short windows takes part in the max
    prec = 0
    for p in range(PRECISION_BITS):
        prec = p
        if _round_half_away(wmax * (1 << (p + 1))) >= (1 << MAX_COEFS_PRECISION):
            break
    out = [(xmin, np.array([max(-32768, min(32767, _round_half_away(v * (1 << prec)))) for v in w], np.int64))
           for xmin, w in rows]
    return out, prec


def _round_half_away(v):
    """Rust f64::round: half away from zero."""
    return int(math.floor(abs(v) + 0.5)) * (1 if v >= 0 else -1)


def _clip8(v, prec):
    v = v >> prec
    return np.clip(v, 0, 255).astype(np.uint8)


def resize(rgb: np.ndarray, S: int, interpolation="bicubic", mode="shortest") -> np.ndarray:
    H, W = rgb.shape[:2]
    x0, y0, x1, y1 = crop_box(W, H, S, mode)
    filt, sup = (_cubic, 2.0) if interpolation == "bicubic" else (_triangle, 1.0)
    ch, ph = _coeffs(W, x0, x1, S, filt, sup)
    cv, pv = _coeffs(H, y0, y1, S, filt, sup)
    need_h = S != W or x0 != 0.0 or x1 != S
    need_v = S != H or y0 != 0.0 or y1 != S
    src = rgb.astype(np.int64)
    if need_h:
        yfirst = cv[0][0]
        ylast = max(ymin + len(k) for ymin, k in cv)
        rows = src[yfirst:ylast]
        tmp = np.empty((ylast - yfirst, S, 3), np.uint8)
        for xx, (xmin, k) in enumerate(ch):
            acc = (rows[:, xmin:xmin + len(k)] * k[None, :, None]).sum(1) + (1 << (ph - 1))
            tmp[:, xx] = _clip8(acc, ph)
        src = tmp.astype(np.int64)
        cv = [(ymin - yfirst, k) for ymin, k in cv]
    if not need_v:
        return src[:S].astype(np.uint8)
    out = np.empty((S, S, 3), np.uint8)
    for yy, (ymin, k) in enumerate(cv):
        acc = (src[ymin:ymin + len(k)] * k[:, None, None]).sum(0) + (1 << (pv - 1))
        out[yy] = _clip8(acc, pv)
    return out


def normalize_pixels(rgb: np.ndarray, mean, std) -> np.ndarray:
    """[S,S,3] u8 -> [3,S,S] f32: (p / 255 - mean[c]) / std[c] in f32 (src/vision.rs:251-256)."""
    x = rgb.astype(np.float32) / np.float32(255.0)
    x = (x - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return np.ascontiguousarray(x.transpose(2, 0, 1))


def preprocess(rgb, S, mean, std, interpolation="bicubic", mode="shortest"):
    return normalize_pixels(resize(rgb, S, interpolation, mode), mean, std)


# ---- resize_with_image (src/vision.rs:200-233): the crate's non-default resize ---------------
# The image crate 0.25.9's imageops::resize (not in this image), restated from its published
# sample.rs in f32 numpy with the crate's operation order (csrc/host/resize_image.cpp is the
# product; test_cpu_preprocess.py checks the two bit for bit, and against Pillow loosely).
F32 = np.float32


def _catmullrom_f32(x):
    b, c = F32(0.0), F32(0.5)
    a = F32(abs(F32(x)))
    if a < F32(1.0):
        k = (F32(12.0) - F32(9.0) * b - F32(6.0) * c) * (a * (a * a)) + \
            (F32(-18.0) + F32(12.0) * b + F32(6.0) * c) * (a * a) + (F32(6.0) - F32(2.0) * b)
    elif a < F32(2.0):
        k = (-b - F32(6.0) * c) * (a * (a * a)) + (F32(6.0) * b + F32(30.0) * c) * (a * a) + \
            (F32(-12.0) * b - F32(48.0) * c) * a + (F32(8.0) * b + F32(24.0) * c)
    else:
        k = F32(0.0)
    return F32(k / F32(6.0))


def _image_kernel(f, x):
    if f == "catmullrom":
        return _catmullrom_f32(x)
    if f == "triangle":
        ax = F32(abs(F32(x)))
        return F32(F32(1.0) - ax) if ax < F32(1.0) else F32(0.0)
    return F32(1.0)


def _image_taps(n_in, n_out, f):
    support = {"catmullrom": 2.0, "triangle": 1.0}.get(f, 0.0)
    ratio = F32(F32(n_in) / F32(n_out))
    sratio = F32(1.0) if ratio < F32(1.0) else ratio
    src_support = F32(F32(support) * sratio)
    taps = []
    for o in range(n_out):
        centre = F32((F32(o) + F32(0.5)) * ratio)
        left = int(math.floor(F32(centre - src_support)))
        left = min(max(left, 0), n_in - 1)
        right = int(math.ceil(F32(centre + src_support)))
        right = min(max(right, left + 1), n_in)
        c = F32(centre - F32(0.5))
        ws = [_image_kernel(f, F32((F32(i) - c) / sratio)) for i in range(left, right)]
        s = F32(0.0)
        for w in ws:
            s = F32(s + w)
        taps.append((left, [F32(w / s) for w in ws]))
    return taps


def _round_half_away_u8(t):
    t = np.clip(t, F32(0.0), F32(255.0)).astype(np.float64)
    fl = np.floor(t)
    return np.where(t - fl >= 0.5, fl + 1, fl).astype(np.uint8)


def image_resize(rgb, nw, nh, f):
    """image::imageops::resize(Rgb<u8>, nw, nh, filter) -> [nh][nw][3] u8."""
    H, W = rgb.shape[:2]
    if (nw, nh) == (W, H):
        return rgb.copy()
    src = rgb.astype(F32)
    tmp = np.empty((nh, W, 3), F32)
    for oy, (left, ws) in enumerate(_image_taps(H, nh, f)):      # vertical_sample
        t = np.zeros((W, 3), F32)
        for i, w in enumerate(ws):
            t = (t + (src[left + i] * w).astype(F32)).astype(F32)
        tmp[oy] = t
    out = np.empty((nh, nw, 3), np.uint8)
    for ox, (left, ws) in enumerate(_image_taps(W, nw, f)):      # horizontal_sample
        t = np.zeros((nh, 3), F32)
        for i, w in enumerate(ws):
            t = (t + (tmp[:, left + i] * w).astype(F32)).astype(F32)
        out[:, ox] = _round_half_away_u8(t)
    return out


def resize_with_image(rgb, S, interpolation="bicubic", resize_mode="shortest"):
    """src/vision.rs:200-233 for an RGB8 image -> [S][S][3] u8."""
    f = {"bicubic": "catmullrom", "bilinear": "triangle"}.get(interpolation, "nearest")
    if resize_mode == "squash":
        return image_resize(rgb, S, S, f)
    H, W = rgb.shape[:2]
    scale = F32(F32(S) / F32(min(W, H)))

    def rnd(v):  # f32::round (half away from zero) then `as u32` (saturating)
        v = float(v)
        r = math.floor(abs(v) + 0.5) * (1 if v >= 0 else -1)
        return max(int(r), 0)
    sw, sh = rnd(F32(F32(W) * scale)), rnd(F32(F32(H) * scale))
    r = image_resize(rgb, sw, sh, f)
    x = rnd(F32(F32(F32(sw) - F32(S)) / F32(2.0)))
    y = rnd(F32(F32(F32(sh) - F32(S)) / F32(2.0)))
    return r[y:y + S, x:x + S].copy()
