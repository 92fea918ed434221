#!/usr/bin/env python3
"""Write the ViT-B/32 vision embeddings of the bench's seeded batch (B = 256) to OUT.npy with the
engine settings of this process's environment; compare two such files with --cmp A B (bit-equal
or not, max |diff|).  For A/B of settings that are read once per process (kernel launch knobs)."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    print(f"bit_equal={np.array_equal(a, b)} max_abs_diff={float(np.abs(a - b).max()):.3g}")
    sys.exit(0 if np.array_equal(a, b) else 1)

import torch  # noqa: E402
from open_clip_inference.engine import Engine  # noqa: E402
from tile_table import WORKLOADS, model_dir  # noqa: E402

cfg, tower, B = WORKLOADS[os.environ.get("WORKLOAD", "b32_vision")]
e = Engine(model_dir(cfg), tower, [0], "bf16", B)
mc = cfg["model_cfg"]
g = torch.Generator(device="cpu").manual_seed(5)
if tower == 0:
    S = mc["vision_cfg"]["image_size"]
    x = torch.randn((B, 3, S, S), generator=g).cuda()
    out = torch.empty((B, mc["embed_dim"]), device="cuda")
    e.embed_pixels_device(x.data_ptr(), B, out.data_ptr(), 0)
else:
    T, V = mc["text_cfg"]["context_length"], mc["text_cfg"]["vocab_size"]
    ids = torch.randint(0, V - 2, (B, T), generator=g, dtype=torch.int64)
    ids[:, -1] = V - 1
    ids = ids.cuda()
    out = torch.empty((B, mc["embed_dim"]), device="cuda")
    e.embed_tokens_device(ids.data_ptr(), B, out.data_ptr(), 0)
torch.cuda.synchronize()
np.save(sys.argv[1], out.cpu().numpy())
e.close()
