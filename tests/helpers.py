"""Shared test helpers: synthetic model dirs, oracle shortcuts, tolerances."""
import json
import os
import tempfile

import numpy as np

from oracle import clip_ref, weights
from oracle.model_spec import (OPENAI_MODEL_CONFIG, TINY_CFG, VIT_B_32_CFG, text_spec_from_cfg,
                               vision_spec_from_cfg)

# north_star: embeddings cosine-equal to the fp32 reference >= 0.9999
COS_TOL = 0.9999


def make_model_dir(cfg=VIT_B_32_CFG, seed=1234, tokenizer_json=None, model_config=None, root=None):
    d = tempfile.mkdtemp(prefix="clipgpu_model_", dir=root)
    with open(os.path.join(d, "open_clip_config.json"), "w") as f:
        json.dump(cfg, f)
    with open(os.path.join(d, "model_config.json"), "w") as f:
        json.dump(model_config or OPENAI_MODEL_CONFIG, f)
    with open(os.path.join(d, "clipgpu_synthetic.json"), "w") as f:
        json.dump({"seed": seed}, f)
    if tokenizer_json is not None:
        with open(os.path.join(d, "tokenizer.json"), "w") as f:
            f.write(tokenizer_json)
    return d


def specs(cfg):
    return vision_spec_from_cfg(cfg["model_cfg"]), text_spec_from_cfg(cfg["model_cfg"])


def normalized_pixels(u8_nhwc, mean, std):
    """normalize_pixels (src/vision.rs:235-259) in numpy f32, HWC -> CHW."""
    x = u8_nhwc.astype(np.float32) / np.float32(255.0)
    x = (x - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return np.ascontiguousarray(x.transpose(0, 3, 1, 2))
