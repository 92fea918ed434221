#!/usr/bin/env python3
"""Per-site MX-fp8 ablation (BASELINE configs[4] "fp8 MFMA weight path"): which GEMM sites can
run in MX-fp8 and keep the north-star cosine bar (>= 0.9999 per row) against the fp32 reference.

For each tower (ViT-B/32 vision + text, DFN5B ViT-H/14-378 vision + text, SO400M-16-SigLIP2-384
vision) and each site split of Engine(mx_sites=...) (c_proj in MX needs c_fc in MX; out_proj,
attention, stems and heads are always bf16) one fp8 engine embeds a seeded batch; the rows are
compared with the fp32 CPU port of the same graph (oracle/torch_cpu.py; SigLIP: oracle/clip_ref.py
in fp32) and with the bf16 engine.  Also times the device-resident forward at a bench-sized batch.
Prints one JSON line per (tower, split).  Test infrastructure: runs on the GPU box.
"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))

from open_clip_inference.engine import Engine  # noqa: E402
from oracle import clip_ref, torch_cpu, weights  # noqa: E402
from oracle.model_spec import (OPENAI_MEAN, OPENAI_MODEL_CONFIG, OPENAI_STD, SIGLIP_MEAN, SIGLIP_STD,  # noqa: E402
                               SO400M_16_SIGLIP2_384_CFG, VIT_B_32_CFG, VIT_H_14_378_CFG, text_spec_from_cfg,
                               vision_spec_from_cfg)

SPLITS = ["", "qkv", "fc", "fc,proj", "qkv,fc", "qkv,fc,proj"]
SEED = 1234


def model_dir(cfg):
    d = tempfile.mkdtemp(prefix="clipgpu_mx_")
    for name, obj in (("open_clip_config.json", cfg), ("model_config.json", OPENAI_MODEL_CONFIG),
                      ("clipgpu_synthetic.json", {"seed": SEED})):
        with open(os.path.join(d, name), "w") as f:
            json.dump(obj, f)
    return d


def cos_rows(a, b):
    return clip_ref.cosine_rows(a, b)


def run(name, cfg, tower, n_check, B_time):
    d = model_dir(cfg)
    v, t = vision_spec_from_cfg(cfg["model_cfg"]), text_spec_from_cfg(cfg["model_cfg"])
    siglip = v.family == "siglip"
    if tower == 0:
        mean, std = (SIGLIP_MEAN, SIGLIP_STD) if siglip else (OPENAI_MEAN, OPENAI_STD)
        u8 = weights.synth_images_u8(17, max(n_check, B_time), v.image_size)
        x = ((u8.astype(np.float32) / np.float32(255) - np.asarray(mean, np.float32)) /
             np.asarray(std, np.float32)).transpose(0, 3, 1, 2).copy()
        P = weights.vision_weights(v, SEED)
        ref = (clip_ref.encode_image(P, v, x[:n_check], dtype=np.float32) if siglip
               else torch_cpu.VisionCPU(P, v)(x[:n_check]))
    else:
        x = weights.synth_token_ids(17, max(n_check, B_time), t.context_length, t.vocab_size, t.vocab_size - 2,
                                    t.vocab_size - 1, random_eot=True)
        ref = torch_cpu.TextCPU(weights.text_weights(t, SEED), t)(x[:n_check])
    d_in = torch.from_numpy(x[:B_time]).cuda()
    s = torch.cuda.current_stream()
    E = cfg["model_cfg"]["embed_dim"]
    out = torch.empty((B_time, E), device="cuda")
    bf16 = None
    for split in [None] + SPLITS:
        if split is None:
            e = Engine(d, tower, [0], "bf16", B_time)
        else:
            e = Engine(d, tower, [0], "fp8", B_time, mx_sites=split)
        got = e.embed_pixels(x[:n_check]) if tower == 0 else e.embed_tokens(x[:n_check])
        fwd = (lambda: e.embed_pixels_device(d_in.data_ptr(), B_time, out.data_ptr(), s.cuda_stream)) if tower == 0 \
            else (lambda: e.embed_tokens_device(d_in.data_ptr(), B_time, out.data_ptr(), s.cuda_stream))
        for _ in range(2):
            fwd()
        torch.cuda.synchronize()
        steps = 5
        t0 = time.perf_counter()
        for _ in range(steps):
            fwd()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        c = cos_rows(got, ref)
        rec = {"tower": name, "engine": "bf16" if split is None else "fp8", "mx_sites": split,
               "cos_vs_fp32_min": round(float(c.min()), 6), "cos_vs_fp32_mean": round(float(c.mean()), 6),
               "meets_0.9999": bool(c.min() >= 0.9999), "rows_checked": n_check,
               "units_per_s": round(B_time / dt, 1), "batch": B_time}
        if bf16 is None:
            bf16 = got
        else:
            rec["cos_vs_bf16_min"] = round(float(cos_rows(got, bf16).min()), 6)
        print(json.dumps(rec), flush=True)
        e.close()


if __name__ == "__main__":
    which = sys.argv[1:] or ["b32_vision", "b32_text", "h14_text", "h14_vision", "so400m_vision"]
    for w in which:
        if w == "b32_vision":
            run(w, VIT_B_32_CFG, 0, 16, 256)
        elif w == "b32_text":
            run(w, VIT_B_32_CFG, 1, 32, 1024)
        elif w == "h14_vision":
            run(w, VIT_H_14_378_CFG, 0, 4, 64)
        elif w == "h14_text":
            run(w, VIT_H_14_378_CFG, 1, 32, 64)
        elif w == "so400m_vision":
            run(w, SO400M_16_SIGLIP2_384_CFG, 0, 2, 128)
