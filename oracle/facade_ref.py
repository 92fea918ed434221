"""Restatement of the Clip facade math (src/clip.rs:79-185) — TEST INFRASTRUCTURE.

compare:      dot(v, t).mul_add(scale, bias)                       (:81-90)
classify:     logits = (T @ v) * scale + bias; sigmoid | softmax; sort desc  (:94-132)
rank_images:  logits = (V @ t) * scale + bias; same                 (:136-170)
softmax:      max-subtracted exp / sum                              (:174-179)
sigmoid:      1 / (1 + exp(-l))                                     (:183-185)
scale / bias default to 1.0 / 0.0; activation defaults to "softmax".
"""
import numpy as np


def softmax(logits):
    x = np.asarray(logits, np.float64)
    e = np.exp(x - x.max())
    return e / e.sum()


def sigmoid(l):
    return 1.0 / (1.0 + np.exp(-np.asarray(l, np.float64)))


def probs(logits, activation):
    return sigmoid(logits) if activation == "sigmoid" else softmax(logits)


def classify(img_emb, text_embs, labels, scale=1.0, bias=0.0, activation="softmax"):
    logits = np.asarray(text_embs, np.float64) @ np.asarray(img_emb, np.float64) * scale + bias
    p = probs(logits, activation)
    order = sorted(range(len(labels)), key=lambda i: -p[i])
    return [(labels[i], float(p[i])) for i in order]


def rank_images(img_embs, text_emb, scale=1.0, bias=0.0, activation="softmax"):
    logits = np.asarray(img_embs, np.float64) @ np.asarray(text_emb, np.float64) * scale + bias
    p = probs(logits, activation)
    order = sorted(range(len(p)), key=lambda i: -p[i])
    return [(i, float(p[i])) for i in order]


def compare(img_emb, text_emb, scale=1.0, bias=0.0):
    return float(np.dot(np.asarray(img_emb, np.float64), np.asarray(text_emb, np.float64)) * scale + bias)


# ---- the reference's f32 arithmetic, bit for bit (test oracle for csrc/host/facade.cpp) ------
# src/clip.rs:79-185 on ndarray 0.17.2 without BLAS (Cargo.toml:14): Array.dot -> ndarray's
# numeric_util::unrolled_dot (eight f32 partial sums); f32::mul_add (one rounding); f32::exp ->
# the platform libm expf (called here through ctypes); Iterator::sum (sequential f32 fold).
import ctypes
import fractions

_libm = ctypes.CDLL("libm.so.6")
_libm.expf.restype = ctypes.c_float
_libm.expf.argtypes = [ctypes.c_float]


def expf(x):
    return np.float32(_libm.expf(float(np.float32(x))))


def unrolled_dot_f32(xs, ys):
    x = np.asarray(xs, np.float32)
    y = np.asarray(ys, np.float32)
    n8 = len(x) // 8 * 8
    p = np.zeros(8, np.float32)
    for i in range(0, n8, 8):
        p = (p + x[i:i + 8] * y[i:i + 8]).astype(np.float32)
    s = np.float32(0)
    for a, b in ((0, 4), (1, 5), (2, 6), (3, 7)):
        s = np.float32(s + np.float32(p[a] + p[b]))
    for i in range(n8, len(x)):
        s = np.float32(s + np.float32(x[i] * y[i]))
    return s


def _round_f32(q: fractions.Fraction) -> np.float32:
    """Round an exact rational to the nearest f32, ties to even."""
    c = np.float32(float(q))
    best = None
    for cand in (np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))):
        if not np.isfinite(cand):
            continue
        d = abs(fractions.Fraction(float(cand)) - q)
        key = (d, int(np.asarray(cand, np.float32).view(np.uint32)) & 1)
        if best is None or key < best[0]:
            best = (key, cand)
    return np.float32(best[1])


def mul_add_f32(a, b, c):
    a, b, c = np.float32(a), np.float32(b), np.float32(c)
    if not (np.isfinite(a) and np.isfinite(b) and np.isfinite(c)):
        return np.float32(np.float64(a) * np.float64(b) + np.float64(c))
    return _round_f32(fractions.Fraction(float(a)) * fractions.Fraction(float(b)) + fractions.Fraction(float(c)))


def softmax_f32(logits):
    x = [np.float32(v) for v in logits]
    m = np.float32(-np.inf)
    for v in x:
        m = np.float32(np.fmax(m, v))
    e = [expf(np.float32(v - m)) for v in x]
    s = np.float32(-0.0)
    for v in e:
        s = np.float32(s + v)
    return [np.float32(v / s) for v in e]


def sigmoid_f32(l):
    return np.float32(np.float32(1.0) / np.float32(np.float32(1.0) + expf(-np.float32(l))))


def scores_f32_exact(embs, query, scale=1.0, bias=0.0, activation="softmax"):
    logits = [mul_add_f32(unrolled_dot_f32(e, query), scale, bias) for e in np.asarray(embs, np.float32)]
    if activation == "logits":
        return logits
    if activation == "sigmoid":
        return [sigmoid_f32(l) for l in logits]
    return softmax_f32(logits)


def classify_f32_exact(img_emb, text_embs, labels, scale=1.0, bias=0.0, activation="softmax"):
    p = scores_f32_exact(text_embs, img_emb, scale, bias, activation)
    order = sorted(range(len(labels)), key=lambda i: -p[i])
    return [(labels[i], float(p[i])) for i in order]


def rank_images_f32_exact(img_embs, text_emb, scale=1.0, bias=0.0, activation="softmax"):
    p = scores_f32_exact(img_embs, text_emb, scale, bias, activation)
    order = sorted(range(len(p)), key=lambda i: -p[i])
    return [(i, float(p[i])) for i in order]
