#!/usr/bin/env python3
"""Per-category serialized ms per step of the bench's text leg (configs[2]: 1024 x 77 ids on the
device), like bench.py --breakdown does for vision.  Runs on the GPU box."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
import bench  # noqa: E402
from open_clip_inference import _lib  # noqa: E402
from open_clip_inference.engine import PROFILE_CATEGORIES, Engine, profile_enable, profile_read  # noqa: E402


def main():
    d = bench.make_model_dir()
    dev = torch.device("cuda:0")
    _, ids = bench.synth_inputs(0, dev)
    te = Engine(d, 1, [0], "bf16", bench.B_TEXT)
    out = torch.empty((bench.B_TEXT, 512), device=dev)
    s = torch.cuda.current_stream()
    step = lambda: te.embed_tokens_device(ids.data_ptr(), bench.B_TEXT, out.data_ptr(), s.cuda_stream)  # noqa: E731
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    steps = 5
    profile_enable(te, PROFILE_CATEGORIES)
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    res = {c: round(profile_read(te, c)[0] / steps, 4) for c in PROFILE_CATEGORIES}
    profile_enable(te, [])
    tiles = (ctypes.c_int * 4)()
    _lib.check(_lib.lib().clipgpu_test_engine_tiles(te._h, tiles))
    lanes = ctypes.c_int()
    _lib.check(_lib.lib().clipgpu_test_engine_lanes(te._h, ctypes.byref(lanes)))
    print(json.dumps({"text_breakdown_ms_per_step": {k: v for k, v in res.items() if v}, "tiles": list(tiles),
                      "lanes": lanes.value, "serialized_total_ms": round(sum(res.values()), 3)}))


if __name__ == "__main__":
    main()
