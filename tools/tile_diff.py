#!/usr/bin/env python3
"""Bitwise comparison of clipgpu_test_gemm across GEMM tiles (diagnostic)."""
import ctypes
import os
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

L = _lib.lib()
rng = np.random.default_rng(0)
for (M, N, K, mode, act) in [(1200, 2304, 768, 0, 0), (1200, 3072, 768, 0, 1), (1200, 768, 768, 1, 0), (1200, 768, 3072, 1, 0),
                             (300, 512, 768, 2, 0)]:
    A = rng.standard_normal((M, K)).astype(np.float32)
    W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    R = rng.standard_normal((M, N)).astype(np.float32)
    outs = {}
    for tile in (1, 2, 3, 4):
        os.environ["CLIPGPU_TEST_TILE"] = str(tile)
        o = np.zeros((M, N), np.float32)
        p = lambda a: a.ctypes.data
        _lib.check(L.clipgpu_test_gemm(0, mode, act, M, N, K, p(A), p(W), p(b), p(R) if mode == 1 else None, p(o)))
        outs[tile] = o
    for tile in (2, 3, 4):
        d = outs[tile] != outs[1]
        if d.any():
            idx = np.argwhere(d)
            print(f"M{M} N{N} K{K} mode{mode}: tile {tile} differs at {d.sum()} of {d.size}; max abs "
                  f"{np.abs(outs[tile] - outs[1]).max():.3g}; first {idx[:4].tolist()} cols mod 16 "
                  f"{sorted(set((idx[:, 1] % 16).tolist()))[:16]}")
        else:
            print(f"M{M} N{N} K{K} mode{mode}: tile {tile} bit-identical")
