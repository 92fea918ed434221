#!/usr/bin/env python3
"""Diagnostic (GPU box): host path vs device path vs repeats, ln_fold on / off, ViT-B/32 max_batch 16,
B = 40 (the gathered-entry-point test's shapes)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from oracle import weights  # noqa: E402
from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, VIT_B_32_CFG, text_spec_from_cfg, vision_spec_from_cfg  # noqa
from open_clip_inference.engine import Engine  # noqa: E402
from tests.helpers import make_model_dir, normalized_pixels  # noqa: E402

d = make_model_dir(VIT_B_32_CFG, seed=1234)
v = vision_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
t = text_spec_from_cfg(VIT_B_32_CFG["model_cfg"])
s = torch.cuda.current_stream()
B = 40
for tower in (0, 1):
    if tower == 0:
        x = normalized_pixels(weights.synth_images_u8(9, B, v.image_size), OPENAI_MEAN, OPENAI_STD)
    else:
        x = weights.synth_token_ids(9, B, t.context_length, t.vocab_size, t.vocab_size - 2, t.vocab_size - 1,
                                    random_eot=True)
    for fold in (None, False):
        for graphs in (None, False):
            e = Engine(d, tower, [0], "bf16", 16, ln_fold=fold, graphs=graphs)
            host = [e.embed_pixels(x) if tower == 0 else e.embed_tokens(x) for _ in range(3)]
            d_in = torch.from_numpy(x).cuda()
            dev = []
            for _ in range(3):
                out = torch.full((B, 512), float("nan"), device="cuda")
                for b0 in range(0, B, 16):
                    n = min(16, B - b0)
                    if tower == 0:
                        e.embed_pixels_device(d_in[b0:].data_ptr(), n, out[b0:].data_ptr(), s.cuda_stream)
                    else:
                        e.embed_tokens_device(d_in[b0:].data_ptr(), n, out[b0:].data_ptr(), s.cuda_stream)
                torch.cuda.synchronize()
                dev.append(out.cpu().numpy())
            rows = lambda a, b: np.where((a != b).any(1))[0].tolist()
            print(f"tower {tower} fold {fold} graphs {graphs}: host repeats {[rows(h, host[0]) for h in host[1:]]} "
                  f"dev repeats {[rows(o, dev[0]) for o in dev[1:]]} host vs dev {rows(host[0], dev[0])}", flush=True)
            e.close()
