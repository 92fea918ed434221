#!/usr/bin/env python3
"""Host-buffer vision path: chunk plans A/B.  One ViT-B/32 bf16 engine at
max_batch 256 (the bench's), u8 [256,224,224,3] host input; per plan (clipgpu_test_host_plan:
chunk bounds, H2D on the copy stream or on the lane streams) the ms per clipgpu_embed_u8 call,
pageable (pinned staging) and caller-registered (clipgpu_host_register), interleaved rounds,
medians; beside the device-resident forward.  HP_BATCHES = n: calls of n x 256 images (the
multi-round path; times per 256-image batch).  copy_stream + 16 / + 32: the multi-round flags of
clipgpu_test_host_plan.  Prints one JSON line per plan.  Runs on the GPU box."""
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402
from open_clip_inference.engine import Engine, host_register, host_unregister  # noqa: E402
from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, VIT_B_32_CFG  # noqa: E402
from tests.helpers import make_model_dir  # noqa: E402

PLANS = [([], 1), ([], 3), ([64], 1), ([64], 3), ([96], 3), ([32], 3)]
if os.environ.get("HP_MODES"):  # e.g. "1,3": the default partition at these copy_stream modes only
    PLANS = [([], int(m)) for m in os.environ["HP_MODES"].split(",")]


def main():
    B = 256
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    nb = int(os.environ.get("HP_BATCHES", "1"))  # batches of 256 per call (multi-round calls: > 1)
    e = Engine(make_model_dir(VIT_B_32_CFG, 1234), 0, [0], "bf16", B)
    g = np.random.default_rng(5)
    x = np.ascontiguousarray(g.integers(0, 256, (B, 224, 224, 3), dtype=np.uint8))
    out = np.empty((B, 512), np.float32)
    if nb > 1:
        x = np.ascontiguousarray(np.concatenate([x] * nb))
        out = np.empty((nb * B, 512), np.float32)
    L = _lib.lib()
    # device-resident reference (the bench's value path)
    d_in = torch.from_numpy(x).cuda()
    d_out = torch.empty((B, 512), device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(3):
        e.embed_u8_device(d_in.data_ptr(), B, OPENAI_MEAN, OPENAI_STD, d_out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        e.embed_u8_device(d_in.data_ptr(), B, OPENAI_MEAN, OPENAI_STD, d_out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    dev_ms = (time.perf_counter() - t0) * 1e3 / 20
    print(json.dumps({"device_resident_ms": round(dev_ms, 3)}), flush=True)
    res = {}
    for r in range(rounds):
        for bounds, cs in PLANS:
            n = len(bounds) + 1 if bounds else 0
            arr = (ctypes.c_int * 4)(*(bounds + [0] * (4 - len(bounds))))
            _lib.check(L.clipgpu_test_host_plan(e._h, n, arr, cs))
            for reg in (0, 1):
                if reg:
                    host_register(x)
                    host_register(out)
                try:
                    e.embed_u8(x, OPENAI_MEAN, OPENAI_STD, out=out)
                    t0 = time.perf_counter()
                    for _ in range(calls):
                        e.embed_u8(x, OPENAI_MEAN, OPENAI_STD, out=out)
                    ms = (time.perf_counter() - t0) * 1e3 / calls
                finally:
                    if reg:
                        host_unregister(x)
                        host_unregister(out)
                res.setdefault((tuple(bounds), cs, reg), []).append(ms / nb)
        print(json.dumps({"round": r}), flush=True)
    for (bounds, cs, reg), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"bounds": list(bounds) or "default", "copy_stream": cs, "registered": reg,
                          "batches_per_call": nb, "ms_per_batch": round(med, 3), "all": [round(t, 3) for t in v],
                          "vs_device": round(dev_ms / med, 3)}), flush=True)


if __name__ == "__main__":
    main()
