#!/usr/bin/env python3
"""Split-K sweep of the N = width GEMMs at one lane's rows (ViT-B/32, batch 128 per lane):
every pipelined tile x K-slices 1/2/3, µs and TFLOP/s per launch (back-to-back launches)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

SHAPES = [("vis_out", 6400, 768, 768), ("vis_c_proj", 6400, 768, 3072), ("patch", 6272, 768, 3072),
          ("vis_out_full", 12800, 768, 768), ("vis_c_proj_full", 12800, 768, 3072)]
L = _lib.lib()
for name, M, N, K in SHAPES:
    for ks in (1, 2, 3):
        if K % (64 * ks) or K // ks < 128:
            continue
        os.environ["CLIPGPU_TEST_KSPLIT"] = str(ks)
        for tile in (1, 2, 3, 4):
            if ks > 1 and tile == 1:
                continue
            us = ctypes.c_double()
            _lib.check(L.clipgpu_test_gemm_bench(0, 1, 0, M, N, K, tile, 20, ctypes.byref(us)))
            tf = 2.0 * M * N * K / (us.value * 1e-6) / 1e12
            print(f"{name:16s} {M:6d}x{N:5d}x{K:5d} ks {ks} tile {tile} {us.value:8.2f} us {tf:7.1f} TF/s", flush=True)
