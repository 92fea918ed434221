#!/usr/bin/env python3
"""Diagnostic (GPU box): the bt kernel (tile 1) vs the pipelined 256x128 (tile 2) on the same
STORE16 GEMM, bf16 and f16, repeated -- do they agree bit for bit?  python tools/bt_diag.py M N K"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from tests.test_gpu_kernels import BF16, F16, round16, run_gemm  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4])
rng = np.random.default_rng(7)
for dt in (BF16, F16):
    A = round16(rng.standard_normal((M, K)), dt)
    W = round16(rng.standard_normal((N, K)) / np.sqrt(K), dt)
    bias = rng.standard_normal(N).astype(np.float32)
    outs = {}
    for t in ("2", "1", "1", "2", "1"):
        os.environ["CLIPGPU_TEST_TILE"] = t
        o = run_gemm(dt, 0, 1, A, W, bias)
        if t in outs:
            print(f"dt {dt} tile {t} repeat equal: {np.array_equal(o, outs[t])}", flush=True)
        else:
            outs[t] = o
    d = outs["1"] != outs["2"]
    print(f"dt {dt}: tile 1 vs 2: {int(d.any(1).sum())} rows differ", flush=True)
