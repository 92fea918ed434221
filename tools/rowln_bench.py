#!/usr/bin/env python3
"""Fused residual GEMM + LayerNorm (gemm_rowln.hip) vs the unfused pair (tiled residual GEMM +
ln_rows_add) at the ViT-B/32 bench shapes: µs per launch, one JSON line per shape.  Runs on the
GPU box; TILES env (comma list) picks the unfused pair's GEMM tiles (default: every tile)."""
import ctypes
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

SHAPES = [  # (name, M, D, K)
    ("vision out_proj+ln_2 B256", 12800, 768, 768),
    ("vision c_proj+ln_1 B256", 12800, 768, 3072),
    ("vision out_proj+ln_2 B128", 6400, 768, 768),
    ("vision c_proj+ln_1 B128", 6400, 768, 3072),
    ("text out_proj+ln_2 B1024x80", 81920, 512, 512),
    ("text c_proj+ln_1 B1024x80", 81920, 512, 2048),
]


PFS = [int(v) for v in os.environ.get("PFS", "0,4,8,12").split(",")]


def main():
    global SHAPES
    if os.environ.get("SHAPES"):  # "M,D,K;M,D,K..."
        SHAPES = [("custom", *map(int, t.split(","))) for t in os.environ["SHAPES"].split(";")]
    L = _lib.lib()
    tiles = [int(t) for t in os.environ.get("TILES", "7,9").split(",")]
    for name, M, D, K in SHAPES:
        us = ctypes.c_double()
        rec = {"shape": name, "M": M, "D": D, "K": K}
        for pf in PFS:
            os.environ["CLIPGPU_ROWLN_PF"] = str(pf)
            _lib.check(L.clipgpu_test_gemm_rowln_bench(0, 0, M, D, K, 20, ctypes.byref(us)))
            rec[f"fused_pf{pf}_us"] = round(us.value, 2)
        os.environ.pop("CLIPGPU_ROWLN_PF", None)
        _lib.check(L.clipgpu_test_gemm_rowln_bench(0, 2, M, D, K, 20, ctypes.byref(us)))
        rec["fused_no_ln_us"] = round(us.value, 2)
        rec["fused_us"] = min(rec[f"fused_pf{pf}_us"] for pf in PFS)
        best = None
        for t in tiles:
            os.environ["CLIPGPU_TEST_TILE"] = str(t)
            _lib.check(L.clipgpu_test_gemm_rowln_bench(0, 1, M, D, K, 20, ctypes.byref(us)))
            rec[f"pair_tile{t}_us"] = round(us.value, 2)
            best = us.value if best is None else min(best, us.value)
        os.environ.pop("CLIPGPU_TEST_TILE", None)
        rec["speedup_vs_best_pair"] = round(best / rec["fused_us"], 3)
        rec["fused_tflops"] = round(2.0 * M * D * K / rec["fused_us"] / 1e6, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
