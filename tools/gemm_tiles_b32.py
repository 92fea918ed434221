#!/usr/bin/env python3
"""Every GEMM tile on the ViT-B/32 trunk shapes at one lane's rows (batch 128 -> 6400 rows)
and at the text lane's rows (512 x 77): µs and TFLOP/s per launch (back-to-back launches)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

NAMES = {1: "128x128", 2: "256x128", 3: "256x256", 4: "128x128p", 5: "128x64p", 6: "64x128p", 7: "160x128p",
         8: "160x64p", 9: "160x128w8", 10: "128x128w8", 11: "192x128w8", 12: "160x256w8"}
if os.environ.get("TILES"):
    NAMES = {int(t): NAMES[int(t)] for t in os.environ["TILES"].split(",")}
SHAPES = [("vis_qkv", 6400, 2304, 768, 0, 0), ("vis_out", 6400, 768, 768, 1, 0), ("vis_c_fc", 6400, 3072, 768, 0, 1),
          ("vis_c_proj", 6400, 768, 3072, 1, 0), ("patch", 6272, 768, 3072, 1, 0),
          ("txt_qkv", 39424, 1536, 512, 0, 0), ("txt_out", 39424, 512, 512, 1, 0),
          ("txt_c_fc", 39424, 2048, 512, 0, 1), ("txt_c_proj", 39424, 512, 2048, 1, 0)]
L = _lib.lib()
for name, M, N, K, epi, act in SHAPES:
    row = []
    for tile in NAMES:
        us = ctypes.c_double()
        _lib.check(L.clipgpu_test_gemm_bench(0, epi, act, M, N, K, tile, 20, ctypes.byref(us)))
        row.append(f"{NAMES[tile]} {us.value:7.2f}us {2.0 * M * N * K / (us.value * 1e-6) / 1e12:6.1f}TF")
    print(f"{name:11s} {M:6d}x{N:5d}x{K:5d} | " + " | ".join(row), flush=True)
    best = min(row, key=lambda r: float(r.split()[1][:-2]))
    print(f"{'':11s} best: {best}", flush=True)
