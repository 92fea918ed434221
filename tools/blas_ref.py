#!/usr/bin/env python3
"""Yardstick only (not product): hipBLASLt bf16 GEMM time via torch.nn.functional.linear on the
trunk shapes, next to clipgpu's own GEMM (clipgpu_test_gemm_bench, autotuned tile = best of 1..3)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

SHAPES = [("vis_qkv", 6400, 2304, 768), ("vis_out", 6400, 768, 768), ("vis_c_fc", 6400, 3072, 768),
          ("vis_c_proj", 6400, 768, 3072), ("vis_c_fc_full", 12800, 3072, 768),
          ("txt_qkv", 39424, 1536, 512), ("txt_c_fc", 39424, 2048, 512), ("txt_c_proj", 39424, 512, 2048),
          ("square4k", 4096, 4096, 4096), ("square8k", 8192, 8192, 8192)]


def t_torch(M, N, K, iters=50):
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        torch.nn.functional.linear(a, w, b)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        torch.nn.functional.linear(a, w, b)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


L = _lib.lib()
for name, M, N, K in SHAPES:
    us = t_torch(M, N, K)
    f = 2.0 * M * N * K
    res = []
    for tile in (1, 2, 3, 4):
        v = ctypes.c_double()
        _lib.check(L.clipgpu_test_gemm_bench(0, 0, 0, M, N, K, tile, 50, ctypes.byref(v)))
        res.append(f"t{tile} {f / v.value / 1e6:6.0f}")
    print(f"{name:14s} {M:6d}x{N:5d}x{K:5d}  hipBLASLt {us:8.2f} us {f / us / 1e6:7.1f} TF | clipgpu TF/s "
          + " ".join(res), flush=True)
