#!/usr/bin/env python3
"""Row-split GEMM experiment (GPU box): a one-lane trunk GEMM (M = 12800) as one launch of its tuned
tile vs two back-to-back launches -- the first M1 rows on a big tile (whole rounds of blocks), the
remaining rows on a smaller tile that fills the last round.  µs per launch pair, one JSON line each."""
import ctypes
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

L = _lib.lib()


def us(epi, act, M, N, K, tile):
    v = ctypes.c_double()
    _lib.check(L.clipgpu_test_gemm_bench(0, epi, act, M, N, K, tile, 20, ctypes.byref(v)))
    return v.value


CASES = [("c_fc", 0, 1, 3072, 768), ("qkv", 0, 0, 2304, 768)]
M = 12800
for name, epi, act, N, K in CASES:
    whole = {t: round(us(epi, act, M, N, K, t), 2) for t in (3, 7, 9, 12)}
    print(json.dumps({"site": name, "M": M, "whole_us": whole}), flush=True)
    for m1 in (256 * 21, 256 * 28, 256 * 40, 256 * 42, 256 * 44):
        for small in (4, 7, 9, 10, 5):
            a = us(epi, act, m1, N, K, 3)
            b = us(epi, act, M - m1, N, K, small)
            print(json.dumps({"site": name, "M1": m1, "big": 3, "small": small, "us": round(a + b, 2),
                              "big_us": round(a, 2), "small_us": round(b, 2)}), flush=True)
