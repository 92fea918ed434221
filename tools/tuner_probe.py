#!/usr/bin/env python3
"""The committed tile table against the timing tuner's picks (clipgpu_options.tuning) for an engine of
the bench workload, interleaved rounds in one process; one JSON line per (variant, round) with the
tiles chosen.  usage: tuner_probe.py vision|text [bf16|fp8]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
import bench  # noqa: E402
from open_clip_inference import _lib  # noqa: E402
from open_clip_inference.engine import Engine  # noqa: E402

tower = sys.argv[1] if len(sys.argv) > 1 else "vision"
dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16"
dev = torch.device("cuda:0")
px, ids = bench.synth_inputs(0, dev)
mdir = bench.make_model_dir()
B = bench.B_VISION if tower == "vision" else bench.B_TEXT
tw = _lib.TOWER_VISION if tower == "vision" else _lib.TOWER_TEXT
engines = {k: Engine(mdir, tw, [0], dtype, B, **v) for k, v in {"table": {}, "tuned": {"tuning": True}}.items()}
out = torch.empty((B, 512), device=dev)
stream = torch.cuda.current_stream()
for rnd in range(3):
    for k, e in engines.items():
        def step():
            if tower == "vision":
                e.embed_pixels_device(px.data_ptr(), B, out.data_ptr(), stream.cuda_stream)
            else:
                e.embed_tokens_device(ids.data_ptr(), B, out.data_ptr(), stream.cuda_stream)
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"tower": tower, "dtype": dtype, "variant": k, "round": rnd,
                          "units_s": round(B * 20 / dt, 1), "info": e.info()}), flush=True)
