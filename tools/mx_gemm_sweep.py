#!/usr/bin/env python3
"""MX-fp8 vs bf16 GEMM timing at the trunk shapes (GPU box): clipgpu_test_gemm_mx_bench /
clipgpu_test_gemm_bench, device-resident random operands, µs per launch and TFLOP/s."""
import ctypes
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
import torch  # noqa: F401,E402  (one HIP runtime per process)
from open_clip_inference import _lib  # noqa: E402

# (label, M, N, K, epi, act): per-lane rows at the BASELINE per-GPU batches
SHAPES = [
    ("h14_qkv", 23360, 3840, 1280, 0, 0), ("h14_fc", 23360, 5120, 1280, 3, 2), ("h14_proj", 23360, 1280, 5120, 1, 0),
    ("so400m_fc", 36864, 4352, 1152, 3, 3), ("so400m_proj", 36864, 1152, 4352, 1, 0),
    ("b32_fc", 6400, 3072, 768, 3, 1), ("b32_proj", 6400, 768, 3072, 1, 0),
]


def main():
    L = _lib.lib()
    us = ctypes.c_double()
    for label, M, N, K, epi, act in SHAPES:
        row = {"shape": label, "M": M, "N": N, "K": K}
        for tile in (2, 3):
            _lib.check(L.clipgpu_test_gemm_mx_bench(epi, act, M, N, K, tile, 10, ctypes.byref(us)))
            row[f"mx_t{tile}_us"] = round(us.value, 1)
            row[f"mx_t{tile}_tflops"] = round(2 * M * N * K / us.value / 1e6, 1)
        bepi = 0 if epi == 3 else epi
        _lib.check(L.clipgpu_test_gemm_bench(0, bepi, act, M, N, K, 0, 10, ctypes.byref(us)))
        row["bf16_auto_us"] = round(us.value, 1)
        row["bf16_tflops"] = round(2 * M * N * K / us.value / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
