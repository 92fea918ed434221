#!/usr/bin/env python3
"""Diagnostic (GPU box): EPI_LNF outputs per tile vs the fp64 LayerNorm-then-Linear reference --
which tiles / rows disagree.  python tools/lnf_diag.py M N K act"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from tests.test_gpu_kernels import BUILT_TILES, BF16, lnf_case, ref_act, run_lnf  # noqa: E402

M, N, K, act = (int(a) for a in sys.argv[1:5])
x, w, gamma, beta, b, wf, cs, bp = lnf_case(M, N, K, M + N + act)
mu = x.mean(1, keepdims=True)
var = ((x - mu) ** 2).mean(1, keepdims=True)
ref = ref_act(act, ((x - mu) / np.sqrt(var + 1e-5) * gamma + beta) @ w.T + b)
outs = {}
for t in [0] + BUILT_TILES + ([100] if M <= 256 else []):
    o = run_lnf(BF16, act, x, wf, cs, bp, 1e-5, t)
    outs[t] = o
    err = np.abs(o - ref)
    bad = np.where(err.max(1) > 0.05 * np.sqrt(np.mean(ref ** 2)))[0]
    print(f"tile {t}: max err {err.max():.4g}, rows off {len(bad)} first {bad[:8].tolist()}", flush=True)
for t, o in outs.items():
    d = np.where((o != outs[0]).any(1))[0]
    print(f"tile {t} vs auto: {len(d)} rows differ, first {d[:8].tolist()}", flush=True)
    if len(d):
        diff = o != outs[0]
        mt, nt = (M + 127) // 128, (N + 127) // 128
        bad = sorted({(i, j) for i in range(mt) for j in range(nt) if diff[i * 128:(i + 1) * 128, j * 128:(j + 1) * 128].any()})
        print(f"  128x128 tiles that differ ({len(bad)}): {bad[:40]}", flush=True)
        i, j = bad[0]
        blk = diff[i * 128:(i + 1) * 128, j * 128:(j + 1) * 128]
        print(f"  tile {bad[0]}: rows {np.where(blk.any(1))[0].tolist()[:20]} cols {np.where(blk.any(0))[0].tolist()[:20]}",
              flush=True)
