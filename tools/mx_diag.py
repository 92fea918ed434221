#!/usr/bin/env python3
"""Diagnose an MX GEMM mismatch: error statistics and the column / row permutation (within
32-blocks) that would explain it.  GPU box: python tools/mx_diag.py [M N K tile]."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))

from oracle import mx_ref  # noqa: E402
from open_clip_inference import _lib as L  # noqa: E402


def main():
    M, N, K, tile = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (128, 128, 128, 3)))
    os.environ["CLIPGPU_TEST_TILE"] = str(tile)
    rng = np.random.default_rng(1)
    for variant in ("unit", "random"):
        if variant == "unit":  # small integers, unit scales: exact products
            A = rng.integers(-2, 3, size=(M, K)).astype(np.float32)
            W = rng.integers(-2, 3, size=(N, K)).astype(np.float32)
            A[:, :32] = A[:, :32]  # keep
        else:
            A = rng.standard_normal((M, K)).astype(np.float32)
            W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
        aq, as_ = mx_ref.quantize_rows(A)
        wq, ws = mx_ref.quantize_rows(W)
        out = np.empty((M, N), np.float32)
        oq = np.empty((M, N), np.uint8)
        os_ = np.empty((M, N // 32), np.uint8)
        L.check(L.lib().clipgpu_test_gemm_mx(0, 2, 0, M, N, K, aq.ctypes.data, as_.ctypes.data, wq.ctypes.data,
                                             ws.ctypes.data, None, None, out.ctypes.data, oq.ctypes.data,
                                             os_.ctypes.data))
        ref = mx_ref.mx_gemm_ref(aq, as_, wq, ws)
        err = np.abs(out - ref)
        print(f"[{variant}] max|ref| {np.abs(ref).max():.4g} max err {err.max():.4g} "
              f"frac exact {(err < 1e-3 * (1 + np.abs(ref))).mean():.4f} ratio out/ref median "
              f"{np.median(out / np.where(ref == 0, 1, ref)):.4g}")
        # column map: for output column j, which reference column matches best (row-wise)?
        cmap = [int(np.argmin(np.abs(out[:, j:j + 1] - ref).sum(0))) for j in range(min(N, 64))]
        print("  out col -> ref col:", cmap)
        rmap = [int(np.argmin(np.abs(out[i:i + 1, :] - ref).sum(1))) for i in range(min(M, 64))]
        print("  out row -> ref row:", rmap)
        if variant == "unit":
            # does any K-permutation fix it? compare with ref computed on K halves / blocks
            for kb in range(K // 32):
                part = mx_ref.dequantize(aq, as_)[:, 32 * kb:32 * kb + 32] @ mx_ref.dequantize(wq, ws)[:, 32 * kb:32 * kb + 32].T
                print(f"  corr(out, block {kb} partial) = {np.corrcoef(out.ravel(), part.ravel())[0, 1]:.3f}")


if __name__ == "__main__":
    main()
