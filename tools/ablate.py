#!/usr/bin/env python3
"""Marginal step-time of each trunk op in the concurrent-lane forward (diagnostic only).

Runs the bench's vision (B = 256) and text (B = 1024 x 77) engines from the ablation build
(`make variant VNAME=ablate VDEFS=-DCLIPGPU_ABLATE`, loaded through CLIPGPU_LIB) and times the
device-resident step with trunk ops skipped (clipgpu_test_ablate mask bits: 0 LayerNorm,
1 attention, 2 out_proj, 3 qkv, 4 c_fc, 5 c_proj).  Masks interleave over ROUNDS rounds in one
process.  The outputs of an ablated step are garbage: only the times mean anything.
One JSON line per (tower, mask, round) to stdout.
"""
import ctypes
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

MASKS = [0, 1, 2, 4, 8, 16, 32, 3, 63]
NAMES = {0: "none", 1: "ln", 2: "attn", 4: "out_proj", 8: "qkv", 16: "c_fc", 32: "c_proj", 3: "ln+attn", 63: "all"}


def main():
    rounds = int(os.environ.get("ABL_ROUNDS", "3"))
    steps = int(os.environ.get("ABL_STEPS", "20"))
    L = _lib.lib()
    ab = L.clipgpu_test_ablate
    ab.argtypes = [ctypes.c_uint]
    ab.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    mdir = bench.make_model_dir()
    px, ids = bench.synth_inputs(0, dev)
    stream = torch.cuda.current_stream(dev)
    towers = os.environ.get("ABL_TOWERS", "vision,text").split(",")
    for tower in towers:
        if tower == "vision":
            eng = Engine(mdir, _lib.TOWER_VISION, [0], "bf16", bench.B_VISION)
            out = torch.empty((bench.B_VISION, 512), device=dev)

            def step():
                eng.embed_pixels_device(px.data_ptr(), bench.B_VISION, out.data_ptr(), stream.cuda_stream)
            units = bench.B_VISION
        else:
            eng = Engine(mdir, _lib.TOWER_TEXT, [0], "bf16", bench.B_TEXT)
            out = torch.empty((bench.B_TEXT, 512), device=dev)

            def step():
                eng.embed_tokens_device(ids.data_ptr(), bench.B_TEXT, out.data_ptr(), stream.cuda_stream)
            units = bench.B_TEXT
        for r in range(rounds):
            for m in MASKS:
                ab(m)
                for _ in range(3):
                    step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    step()
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                print(json.dumps({"tower": tower, "round": r, "mask": m, "skipped": NAMES[m],
                                  "ms_per_step": round(dt * 1e3 / steps, 4),
                                  "units_s": round(units * steps / dt, 1)}), flush=True)
        ab(0)
        eng.close()


if __name__ == "__main__":
    main()
