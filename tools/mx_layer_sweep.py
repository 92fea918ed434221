#!/usr/bin/env python3
"""Per-layer MX-fp8 sensitivity sweep: which transformer layers of an fp8
engine can run their MX sites in MX-fp8 (clipgpu_options.mx_layers) and keep the north-star bar
(min row cosine >= 0.9999 against the fp32 graph of the same seeded weights).

For each tower and MX site split:
  1. one fp8 engine per layer l with mx_layers = 1 << l (every other layer all-bf16): the cosine
     deficit 1 - min cos that layer alone costs;
  2. greedy: layers in order of increasing deficit are added while the whole mask still meets
     the bar (each prefix measured, not summed), and the largest passing mask is timed
     device-resident at the bench batch beside the bf16 engine and the all-layer split.
Prints one JSON line per measurement.  Test infrastructure: runs on the GPU box.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))

from open_clip_inference.engine import Engine  # noqa: E402
from oracle import torch_cpu, weights  # noqa: E402
from oracle.model_spec import (OPENAI_MEAN, OPENAI_STD, VIT_B_32_CFG, VIT_H_14_378_CFG,  # noqa: E402
                               text_spec_from_cfg, vision_spec_from_cfg)
from tools.mx_ablation import SEED, cos_rows, model_dir  # noqa: E402

BAR = 0.9999


def emit(**rec):
    print(json.dumps(rec), flush=True)


def sweep(name, cfg, tower, n_check, B_time, splits):
    d = model_dir(cfg)
    v, t = vision_spec_from_cfg(cfg["model_cfg"]), text_spec_from_cfg(cfg["model_cfg"])
    layers = (v if tower == 0 else t).layers
    if tower == 0:
        u8 = weights.synth_images_u8(17, max(n_check, B_time), v.image_size)
        x = ((u8.astype(np.float32) / np.float32(255) - np.asarray(OPENAI_MEAN, np.float32)) /
             np.asarray(OPENAI_STD, np.float32)).transpose(0, 3, 1, 2).copy()
        ref = torch_cpu.VisionCPU(weights.vision_weights(v, SEED), v)(x[:n_check])
    else:
        x = weights.synth_token_ids(17, max(n_check, B_time), t.context_length, t.vocab_size, t.vocab_size - 2,
                                    t.vocab_size - 1, random_eot=True)
        ref = torch_cpu.TextCPU(weights.text_weights(t, SEED), t)(x[:n_check])

    def check(dtype, **kw):
        e = Engine(d, tower, [0], dtype, n_check, **kw)
        got = e.embed_pixels(x[:n_check]) if tower == 0 else e.embed_tokens(x[:n_check])
        e.close()
        return float(cos_rows(got, ref).min())

    def timed(dtype, **kw):
        e = Engine(d, tower, [0], dtype, B_time, **kw)
        d_in = torch.from_numpy(x[:B_time]).cuda()
        out = torch.empty((B_time, cfg["model_cfg"]["embed_dim"]), device="cuda")
        s = torch.cuda.current_stream()
        fwd = (lambda: e.embed_pixels_device(d_in.data_ptr(), B_time, out.data_ptr(), s.cuda_stream)) if tower == 0 \
            else (lambda: e.embed_tokens_device(d_in.data_ptr(), B_time, out.data_ptr(), s.cuda_stream))
        for _ in range(3):
            fwd()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):  # best of 3 windows of 5 forwards
            t0 = time.perf_counter()
            for _ in range(5):
                fwd()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / 5)
        e.close()
        return round(B_time / best, 1)

    emit(tower=name, engine="bf16", cos_min=round(check("bf16"), 7), units_per_s=timed("bf16"), batch=B_time)
    for split in splits:
        t0 = time.time()
        full = check("fp8", mx_sites=split)
        emit(tower=name, engine="fp8", mx_sites=split, mx_layers="all", cos_min=round(full, 7),
             units_per_s=timed("fp8", mx_sites=split), batch=B_time)
        deficit = {}
        for l in range(layers):
            c = check("fp8", mx_sites=split, mx_layers=1 << l)
            deficit[l] = 1.0 - c
            emit(tower=name, mx_sites=split, layer=l, cos_min=round(c, 7), deficit=float(f"{1.0 - c:.3e}"))
        order = sorted(range(layers), key=lambda l: deficit[l])
        mask, chosen, last = 0, [], None
        for l in order:
            c = check("fp8", mx_sites=split, mx_layers=mask | (1 << l))
            emit(tower=name, mx_sites=split, greedy_add=l, n_layers=len(chosen) + 1, cos_min=round(c, 7))
            if c < BAR:
                break
            mask |= 1 << l
            chosen.append(l)
            last = c
        rec = {"tower": name, "mx_sites": split, "greedy_layers": sorted(chosen), "mx_layers_mask": mask,
               "cos_min": None if last is None else round(last, 7), "sweep_s": round(time.time() - t0, 1)}
        if mask:
            rec["units_per_s"] = timed("fp8", mx_sites=split, mx_layers=mask)
            rec["batch"] = B_time
        emit(**rec)


if __name__ == "__main__":
    which = sys.argv[1:] or ["b32_text", "h14_text"]
    for w in which:
        if w == "b32_text":
            sweep(w, VIT_B_32_CFG, 1, 64, 1024, ["qkv,fc,proj", "fc,proj", "qkv"])
        elif w == "h14_text":
            sweep(w, VIT_H_14_378_CFG, 1, 32, 64, ["qkv,fc,proj", "fc,proj"])
        elif w == "b32_vision":
            sweep(w, VIT_B_32_CFG, 0, 16, 256, ["qkv,fc,proj", "fc,proj"])
