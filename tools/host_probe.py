#!/usr/bin/env python3
"""Host-side rates on the GPU box (one JSON line each): host copy (one thread / the copy pool; into
malloc'd / pinned memory), then the decoded-image entry point at 224x224 and 640x480 with the u8 host
path beside it.  Run under rocprofv3 --kernel-trace to see the resize kernels' share."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

L = _lib.lib()
for mb in (38.5, 118.0):
    n = int(mb * 2 ** 20) // 64 * 64
    for mode, name in ((0, "memcpy"), (1, "pool"), (2, "memcpy_pinned"), (3, "pool_pinned")):
        us = ctypes.c_double()
        _lib.check(L.clipgpu_test_host_copy(n, mode, 5, ctypes.byref(us)))
        print(json.dumps({"host_copy": name, "MB": mb, "us": round(us.value, 1), "GB_s": round(n / us.value / 1e3, 2)}),
              flush=True)

import bench  # noqa: E402
from open_clip_inference.engine import Engine  # noqa: E402
e = Engine(bench.make_model_dir(), 0, [0], "bf16", 256)
g = np.random.default_rng(77)
u8 = g.integers(0, 256, (256, 224, 224, 3), dtype=np.uint8)
dec224 = [u8[i] for i in range(256)]
dec640 = [g.integers(0, 256, (480, 640, 3), dtype=np.uint8) for _ in range(256)]
mean, std = bench.CFG["preprocess_cfg"]["mean"], bench.CFG["preprocess_cfg"]["std"]
for name, fn in (("u8_pageable", lambda: e.embed_u8(u8, mean, std)), ("rgb8_224", lambda: e.embed_images_rgb8(dec224)),
                 ("rgb8_640x480", lambda: e.embed_images_rgb8(dec640))):
    fn()
    t0 = time.perf_counter()
    for _ in range(5):
        fn()
    dt = (time.perf_counter() - t0) / 5
    print(json.dumps({"leg": name, "ms_per_call": round(dt * 1e3, 3), "images_s": round(256 / dt, 1)}), flush=True)
e.close()

# Why bench.py's host legs read slower than the legs above: the same call on an
# array torch allocated, and right after a multi-threaded torch CPU op (its OpenMP workers spin-wait
# on the box's 16-CPU quota beside the copy pool's threads).
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch
    e = Engine(bench.make_model_dir(), 0, [0], "bf16", 256)
    tu8 = torch.from_numpy(u8.copy()).contiguous().numpy()
    cases = [("numpy", u8), ("torch_alloc", tu8)]
    for name, arr in cases:
        e.embed_u8(arr, mean, std)
        t0 = time.perf_counter()
        for _ in range(5):
            e.embed_u8(arr, mean, std)
        dt = (time.perf_counter() - t0) / 5
        print(json.dumps({"leg": "u8_pageable_" + name, "ms_per_call": round(dt * 1e3, 3)}), flush=True)
    x = torch.randn(2048, 2048)
    for _ in range(3):
        (x @ x).sum()
    t0 = time.perf_counter()
    for _ in range(5):
        (x @ x).sum()
        e.embed_u8(u8, mean, std)
    dt = (time.perf_counter() - t0) / 5
    print(json.dumps({"leg": "u8_pageable_after_torch_op", "ms_per_call_incl_op": round(dt * 1e3, 3)}), flush=True)
    t0 = time.perf_counter()
    for _ in range(5):
        (x @ x).sum()
    print(json.dumps({"torch_op_ms": round((time.perf_counter() - t0) / 5 * 1e3, 3)}), flush=True)
    e.close()
