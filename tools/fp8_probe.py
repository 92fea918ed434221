#!/usr/bin/env python3
"""fp8 (MX) vision engine variants at the bench workload (256 images, device-resident): the default
(MX tile heuristic) against the timing tuner's picks (clipgpu_options.tuning) and lane counts,
interleaved rounds in one process; one JSON line per (variant, round) with the tiles chosen."""
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

dev = torch.device("cuda:0")
px = bench.synth_inputs(0, dev)
px = px[0] if isinstance(px, tuple) else px
mdir = bench.make_model_dir()
variants = {"default": {}, "tuned": {"tuning": True}, "lanes1": {"lanes": 1}, "tuned_lanes1": {"tuning": True, "lanes": 1}}
engines = {k: Engine(mdir, _lib.TOWER_VISION, [0], "fp8", bench.B_VISION, **v) for k, v in variants.items()}
out = torch.empty((bench.B_VISION, 512), device=dev)
stream = torch.cuda.current_stream()
for rnd in range(3):
    for k, e in engines.items():
        for _ in range(5):
            e.embed_pixels_device(px.data_ptr(), bench.B_VISION, out.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            e.embed_pixels_device(px.data_ptr(), bench.B_VISION, out.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"variant": k, "round": rnd, "images_s": round(bench.B_VISION * 20 / dt, 1),
                          "info": e.info()}), flush=True)
