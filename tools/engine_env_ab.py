#!/usr/bin/env python3
"""Interleaved A/B of engine settings that are read at engine creation (environment variables),
in one process: one engine per setting, built with that setting's variables set, then the
device-resident forwards timed round-robin (median of rounds), plus a bit-equality check of the
embeddings of every engine against the first one.

usage: python tools/engine_env_ab.py [--workload b32_vision] [--rounds 9] "" "CLIPGPU_GEMM_XPF=1" ...
(an empty setting is the default engine)
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from open_clip_inference.engine import Engine  # noqa: E402
from tile_table import WORKLOADS, model_dir  # noqa: E402


def build(d, tower, B, setting):
    kv = dict(s.split("=", 1) for s in setting.split() if s)
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    try:
        return Engine(d, tower, [0], "bf16", B)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="b32_vision")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("settings", nargs="+")
    args = ap.parse_args()
    cfg, tower, B = WORKLOADS[args.workload]
    d = model_dir(cfg)
    mc = cfg["model_cfg"]
    engines = [(s or "default", build(d, tower, B, s)) for s in args.settings]
    s = torch.cuda.Stream()  # a real stream handle (the engine forks from / joins back to it)
    torch.cuda.set_stream(s)
    torch.manual_seed(0)
    if tower == 0:
        S = mc["vision_cfg"]["image_size"]
        x = torch.randn((B, 3, S, S), device="cuda")
        fwd = lambda e, o: e.embed_pixels_device(x.data_ptr(), B, o.data_ptr(), s.cuda_stream)  # noqa: E731
    else:
        T, V = mc["text_cfg"]["context_length"], mc["text_cfg"]["vocab_size"]
        ids = torch.randint(0, V - 2, (B, T), device="cuda", dtype=torch.int64)
        ids[:, -1] = V - 1
        fwd = lambda e, o: e.embed_tokens_device(ids.data_ptr(), B, o.data_ptr(), s.cuda_stream)  # noqa: E731
    outs = {k: torch.empty((B, mc["embed_dim"]), device="cuda") for k, _ in engines}
    for k, e in engines:
        for _ in range(3):
            fwd(e, outs[k])
    torch.cuda.synchronize()
    ref = outs[engines[0][0]]
    times = {k: [] for k, _ in engines}
    for _ in range(args.rounds):
        for k, e in engines:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                fwd(e, outs[k])
            torch.cuda.synchronize()
            times[k].append((time.perf_counter() - t0) * 1e3 / 10)
    for k, e in engines:
        tiles, lanes, _ = e.info()
        med = statistics.median(times[k])
        print(json.dumps({"workload": args.workload, "batch": B, "setting": k, "tiles": tiles, "lanes": lanes,
                          "ms_median": round(med, 4), "ms_min": round(min(times[k]), 4),
                          "units_per_s": round(B / med * 1e3, 1),
                          "bit_equal_to_first": bool(torch.equal(outs[k], ref))}), flush=True)
        e.close()


if __name__ == "__main__":
    main()
