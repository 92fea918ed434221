#!/usr/bin/env python3
"""Regenerate / check the committed tile table (engine.hip table_tiles) on one MI355X.

For each BASELINE workload (per-GPU batch), builds engines with
  * the committed table (lanes = 1, the default),
  * the committed table with 2 lanes,
  * the creation-time timing tuner (clipgpu_options.tuning = 1), `--tuned` times,
and times their device-resident forwards interleaved (round-robin, median of rounds), printing one
JSON line per engine: its tiles, lanes and ms per forward.  A tuner pick that beats the table by
more than the spread, consistently, is a candidate for a table entry.

usage: python tools/tile_table.py [--rounds 7] [--tuned 2] [--only b32_vision,b32_text]
"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

import torch  # noqa: F401  (one HIP runtime per process: torch before the native lib)

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))

from open_clip_inference.engine import Engine  # noqa: E402
from oracle.model_spec import (OPENAI_MODEL_CONFIG, SO400M_16_SIGLIP2_384_CFG, VIT_B_32_CFG,  # noqa: E402
                               VIT_H_14_378_CFG)

WORKLOADS = {
    "b32_vision": (VIT_B_32_CFG, 0, 256),
    "b32_text": (VIT_B_32_CFG, 1, 1024),
    "so400m_vision": (SO400M_16_SIGLIP2_384_CFG, 0, 128),
    "h14_vision": (VIT_H_14_378_CFG, 0, 64),
    "h14_text": (VIT_H_14_378_CFG, 1, 64),
}


def model_dir(cfg):
    d = tempfile.mkdtemp(prefix="clipgpu_tiles_")
    for name, obj in (("open_clip_config.json", cfg), ("model_config.json", OPENAI_MODEL_CONFIG),
                      ("clipgpu_synthetic.json", {"seed": 7})):
        with open(os.path.join(d, name), "w") as f:
            json.dump(obj, f)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--tuned", type=int, default=2)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    names = [n for n in WORKLOADS if not args.only or n in args.only.split(",")]
    for name in names:
        cfg, tower, B = WORKLOADS[name]
        d = model_dir(cfg)
        mc = cfg["model_cfg"]
        engines = [("table", Engine(d, tower, [0], "bf16", B)), ("table_2lanes", Engine(d, tower, [0], "bf16", B, lanes=2))]
        for i in range(args.tuned):
            engines.append((f"tuned{i}", Engine(d, tower, [0], "bf16", B, tuning=True)))
        out = torch.empty((B, mc["embed_dim"]), device="cuda")
        s = torch.cuda.current_stream()
        if tower == 0:
            S = mc["vision_cfg"]["image_size"]
            x = torch.randn((B, 3, S, S), device="cuda")
            fwd = lambda e: e.embed_pixels_device(x.data_ptr(), B, out.data_ptr(), s.cuda_stream)  # noqa: E731
        else:
            T, V = mc["text_cfg"]["context_length"], mc["text_cfg"]["vocab_size"]
            ids = torch.randint(0, V - 2, (B, T), device="cuda", dtype=torch.int64)
            ids[:, -1] = V - 1
            fwd = lambda e: e.embed_tokens_device(ids.data_ptr(), B, out.data_ptr(), s.cuda_stream)  # noqa: E731
        times = {k: [] for k, _ in engines}
        for _, e in engines:
            for _ in range(3):
                fwd(e)
        torch.cuda.synchronize()
        # wall clock around a device-wide synchronize: a multi-lane engine forks its lanes onto
        # its own streams, so events recorded on the caller's stream do not bracket the work
        for _ in range(args.rounds):
            for k, e in engines:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5):
                    fwd(e)
                torch.cuda.synchronize()
                times[k].append((time.perf_counter() - t0) * 1e3 / 5)
        for k, e in engines:
            tiles, lanes, _ = e.info()
            med = statistics.median(times[k])
            print(json.dumps({"workload": name, "batch": B, "engine": k, "tiles": tiles, "lanes": lanes,
                              "ms_median": round(med, 4), "ms_min": round(min(times[k]), 4),
                              "units_per_s": round(B / med * 1e3, 1)}), flush=True)
            e.close()


if __name__ == "__main__":
    main()
