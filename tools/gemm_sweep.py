#!/usr/bin/env python3
"""GEMM tile sweep on the GPU: every hot-path GEMM shape of ViT-B/32 (batch 256) and
the text tower (batch 1024 x 77) x every tile config; prints µs and TFLOP/s."""
import json
import os
import sys
import ctypes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

SHAPES = [  # name, M, N, K, epi, act
    ("vis_qkv", 12800, 2304, 768, 0, 0), ("vis_out", 12800, 768, 768, 1, 0),
    ("vis_c_fc", 12800, 3072, 768, 0, 1), ("vis_c_proj", 12800, 768, 3072, 1, 0),
    ("txt_qkv", 78848, 1536, 512, 0, 0), ("txt_out", 78848, 512, 512, 1, 0),
    ("txt_c_fc", 78848, 2048, 512, 0, 1), ("txt_c_proj", 78848, 512, 2048, 1, 0),
    ("square4k", 4096, 4096, 4096, 2, 0),
]
L = _lib.lib()
rows = []
for name, M, N, K, epi, act in SHAPES:
    for tile in (1, 2, 3, 4, 5):
        us = ctypes.c_double()
        _lib.check(L.clipgpu_test_gemm_bench(0, epi, act, M, N, K, tile, 20, ctypes.byref(us)))
        tf = 2.0 * M * N * K / (us.value * 1e-6) / 1e12
        rows.append({"gemm": name, "M": M, "N": N, "K": K, "tile": ["", "128x128", "256x128", "256x256", "ring256", "ring128"][tile],
                     "us": round(us.value, 2), "tflops": round(tf, 1)})
        print(f"{name:12s} {M:6d}x{N:5d}x{K:5d} tile {rows[-1]['tile']:8s} {us.value:9.2f} us {tf:7.1f} TF/s",
              flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "gemm_sweep.json"), "w") as f:
    json.dump(rows, f, indent=1)
