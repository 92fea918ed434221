"""MX-fp8 restatement for the fp8 weight path -- TEST INFRASTRUCTURE (only tests/, smoke()
and bench.py's cpu_baseline import oracle/).

BASELINE.json configs[4] asks for an "fp8 MFMA weight path" (DFN5B ViT-H/14-378).  The
reference itself has no fp8 arithmetic: its ONNX graphs run in f32 (src/onnx.rs:7-47,
pull_onnx.py:53-68), so this module restates OUR format, not the reference's: the parity of
the fp8 path with the reference is reported as the measured cosine against the f32 oracle
(clip_ref.py), which is expected to fall short of the 0.9999 bar (SURVEY.md §7 risk notes).

Format (OCP Microscaling v1.0 "MXFP8 E4M3"): a row of K elements is split into blocks of 32
consecutive elements; each block stores one E8M0 scale byte (2^(byte - 127)) and 32 OCP
e4m3fn elements (bias 7, no infinities, 0x7F / 0xFF are NaN, max 448).  Block exponent rule
(kernels/common.hpp mx_exp): the smallest e with amax <= 448 * 2^e, so no element saturates
(the OCP spec's floor(log2 amax) - 8 would clip the top of the block), computed from the f32
bits of amax; elements are f32(x * 2^-e) rounded to nearest-even e4m3.

The e4m3 encoder was pinned against the gfx950 v_cvt_pk_fp8_f32 instruction on every e4m3
value, every midpoint between neighbours and out-of-range inputs (tools/mx_probe.hip: 0
mismatches, saturating to 448).
"""
from __future__ import annotations

import numpy as np


def e4m3_decode_table() -> np.ndarray:
    """float64 value of each of the 256 e4m3fn codes (NaN for 0x7F / 0xFF)."""
    v = np.arange(256)
    s = np.where(v >> 7, -1.0, 1.0)
    e = (v >> 3) & 15
    m = v & 7
    mag = np.where(e == 0, np.ldexp(m.astype(np.float64), -9), np.ldexp(1.0 + m / 8.0, e - 7))
    out = s * mag
    out[(v & 0x7F) == 0x7F] = np.nan
    return out


_DEC = e4m3_decode_table()
_POS = _DEC[:127]  # codes 0x00 .. 0x7E, ascending


def e4m3_encode(y: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even e4m3fn codes of float32 values (saturating at +-448)."""
    y = np.asarray(y, np.float32)
    a = np.abs(y).astype(np.float64)
    hi = np.clip(np.searchsorted(_POS, a, side="left"), 0, 126)
    lo = np.clip(hi - 1, 0, 126)
    dlo = a - _POS[lo]
    dhi = _POS[hi] - a
    pick_hi = (dhi < dlo) | ((dhi == dlo) & (hi % 2 == 0))
    code = np.where(pick_hi, hi, lo)
    code = np.where(a >= 448.0, 126, code)
    return (code | np.where(np.signbit(y), 0x80, 0)).astype(np.uint8)


def mx_exp(amax: np.ndarray) -> np.ndarray:
    """Block exponent from the f32 bits of amax (common.hpp mx_exp)."""
    b = np.asarray(amax, np.float32).view(np.uint32).astype(np.int64)
    be = b >> 23
    e = be - 135 + ((b & 0x7FFFFF) > 0x600000)
    e = np.where(be == 0, -127, e)
    return np.clip(e, -127, 127)


def quantize_rows(x: np.ndarray):
    """f32 [R][C] (C % 32 == 0) -> (e4m3 codes uint8 [R][C], E8M0 scales uint8 [R][C/32])."""
    x = np.asarray(x, np.float32)
    R, C = x.shape
    assert C % 32 == 0
    xb = x.reshape(R, C // 32, 32)
    e = mx_exp(np.abs(xb).max(-1))
    inv = np.ldexp(np.float32(1.0), -e).astype(np.float32)  # 2^-e exactly
    q = e4m3_encode(xb * inv[..., None])
    return q.reshape(R, C), (e + 127).astype(np.uint8)


def dequantize(q: np.ndarray, s: np.ndarray) -> np.ndarray:
    """float64 values of an MX-fp8 matrix."""
    R, C = q.shape
    v = _DEC[q].reshape(R, C // 32, 32) * np.ldexp(1.0, s.astype(np.int64) - 127)[..., None]
    return v.reshape(R, C)


def mx_gemm_ref(aq, as_, wq, ws, bias=None):
    """float64 A . W^T (+ bias) of MX operands."""
    out = dequantize(aq, as_) @ dequantize(wq, ws).T
    if bias is not None:
        out = out + np.asarray(bias, np.float64)
    return out
