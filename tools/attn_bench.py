#!/usr/bin/env python3
"""Attention kernels alone at the per-lane shapes of the BASELINE configs (GPU box): µs per
launch and TFLOP/s (4*N^2*hd per (image, head); causal counted dense)."""
import ctypes
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
import torch  # noqa: F401,E402
from open_clip_inference import _lib  # noqa: E402

CASES = [("h14_vision", 32, 730, 16, 80, 0), ("so400m_vision", 64, 576, 16, 72, 0), ("h14_text", 32, 77, 16, 64, 1),
         ("b32_vision", 128, 50, 12, 64, 0), ("b32_text", 512, 77, 8, 64, 1),
         ("b32_vision_1lane", 256, 50, 12, 64, 0), ("b32_text_1lane", 1024, 77, 8, 64, 1)]
if os.environ.get("ATTN_LAYOUT_PROBE"):  # the same workgroups and bytes with one head per row: each
    # workgroup's rows then sit 3 x 128 B apart instead of 3 x 768 x 2 B (the head-major-layout question)
    CASES = [("b32_vision", 128, 50, 12, 64, 0), ("b32_vision_h1", 1536, 50, 1, 64, 0),
             ("b32_text", 512, 77, 8, 64, 1), ("b32_text_h1", 4096, 77, 1, 64, 1)] * 2

L = _lib.lib()
us = ctypes.c_double()
for name, B, N, H, HD, causal in CASES:
    _lib.check(L.clipgpu_test_attention_bench(0, B, N, H, HD, causal, 20, ctypes.byref(us)))
    fl = 4.0 * B * H * N * N * HD
    hbm = 2.0 * B * N * H * HD * 4  # qkv read (3 x) + out write (1 x), 16-bit
    print(json.dumps({"case": name, "B": B, "N": N, "H": H, "hd": HD, "us": round(us.value, 1),
                      "tflops": round(fl / us.value / 1e6, 1), "hbm_gbs": round(hbm / us.value / 1e3, 1)}), flush=True)
