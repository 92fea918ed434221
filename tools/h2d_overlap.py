#!/usr/bin/env python3
"""Does a concurrent host-to-device copy slow the device-resident forward?  The multi-round host
path (engine.hip run_host_shard) runs round i + 1's H2D (38.5 MB of u8 for 256 images) under round
i's forwards, and each of its rounds is ~8 % slower than the device-resident call.
ViT-B/32 bf16 at max_batch 256, u8 input already on the device; per setting the ms per call,
interleaved rounds, medians:
  plain   -- the device-resident call alone (the bench's value path);
  h2d     -- the same call with a 38.5 MB pinned H2D issued on a side stream before each call;
  d2d     -- the same with a 38.5 MB device-to-device copy instead (HBM traffic, no PCIe).
Prints one JSON line per setting.  Runs on the GPU box."""
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
from open_clip_inference.engine import Engine  # noqa: E402
from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, VIT_B_32_CFG  # noqa: E402
from tests.helpers import make_model_dir  # noqa: E402


def main():
    B = 256
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    e = Engine(make_model_dir(VIT_B_32_CFG, 1234), 0, [0], "bf16", B)
    g = np.random.default_rng(5)
    x = np.ascontiguousarray(g.integers(0, 256, (B, 224, 224, 3), dtype=np.uint8))
    d_in = torch.from_numpy(x).cuda()
    d_out = torch.empty((B, 512), device="cuda")
    h_buf = torch.from_numpy(x.copy()).pin_memory()
    d_buf = torch.empty_like(d_in)
    d_src = d_in.clone()
    s = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def call(extra):
        if extra == "h2d":
            with torch.cuda.stream(side):
                d_buf.copy_(h_buf, non_blocking=True)
        elif extra == "d2d":
            with torch.cuda.stream(side):
                d_buf.copy_(d_src, non_blocking=True)
        e.embed_u8_device(d_in.data_ptr(), B, OPENAI_MEAN, OPENAI_STD, d_out.data_ptr(), s.cuda_stream)

    res = {}
    for extra in ("plain", "h2d", "d2d"):
        for _ in range(3):
            call(extra)
    torch.cuda.synchronize()
    for _ in range(rounds):
        for extra in ("plain", "h2d", "d2d"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                call(extra)
            torch.cuda.synchronize()
            res.setdefault(extra, []).append((time.perf_counter() - t0) * 1e3 / iters)
    # the copies alone
    for extra, src in (("h2d_alone", h_buf), ("d2d_alone", d_src)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            d_buf.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        res[extra] = [(time.perf_counter() - t0) * 1e3 / iters]
    for k, v in res.items():
        print(json.dumps({"setting": k, "ms": round(statistics.median(v), 3), "all": [round(t, 3) for t in v]}))


if __name__ == "__main__":
    main()
