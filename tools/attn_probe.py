#!/usr/bin/env python3
"""Runs the attention kernels alone on the large-model shapes (for rocprofv3 --pmc passes):
SO400M-384 (576 tokens, 16 heads x 72) and ViT-H/14-378 (730 tokens, 16 x 80), batch 16."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

L = _lib.lib()
for N, H, HD in ((576, 16, 72), (730, 16, 80)):
    B = 16
    qkv = np.random.default_rng(0).standard_normal((B * N, 3 * H * HD)).astype(np.float32)
    out = np.empty((B * N, H * HD), np.float32)
    for _ in range(3):
        _lib.check(L.clipgpu_test_attention(0, B, N, H, HD, 0, qkv.ctypes.data, out.ctypes.data))
print("ok")
