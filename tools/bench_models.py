#!/usr/bin/env python3
"""Throughput of the BASELINE.json large configs and of the host-buffer path (1 GPU).

Not the bench.py contract line: configs[3] / configs[4] are parity-test cases there.  Reported
here per GPU at the per-GPU share of the BASELINE batch (SO400M-16-SigLIP2-384 vision 1024 / 8 =
128 images, DFN5B ViT-H/14-378 vision + text 512 / 8 = 64), device-resident inputs, seeded
weights, plus ViT-B/32 through the HOST entry points (u8 / f32 host buffers, pinned staging,
H2D + D2H included: the PCIe-inclusive rate SURVEY.md §8d asks to report beside the device one).
Prints one JSON line per measurement.
"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime per process: torch before the native lib)

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))

from open_clip_inference import _lib  # noqa: E402
from open_clip_inference.engine import Engine  # noqa: E402
from oracle.model_spec import (OPENAI_MODEL_CONFIG, SO400M_16_SIGLIP2_384_CFG, VIT_B_32_CFG,  # noqa: E402
                               VIT_H_14_378_CFG)

# so400m_text: SigLIP2 text tower, 64 tokens x 27 layers x 2 (4 D^2 + 2 D MLP) + attention + projection
GFLOP = {"so400m_vision": 518.9, "h14_vision": 1007.0, "h14_text": 47.1, "b32_vision": 8.818, "so400m_text": 53.1}


def model_dir(cfg):
    d = tempfile.mkdtemp(prefix="clipgpu_models_")
    for name, obj in (("open_clip_config.json", cfg), ("model_config.json", OPENAI_MODEL_CONFIG),
                      ("clipgpu_synthetic.json", {"seed": 7})):
        with open(os.path.join(d, name), "w") as f:
            json.dump(obj, f)
    return d


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def device_leg(name, cfg, tower, B, steps=6, warmup=2, dtype="bf16", mx_sites=None, lanes=0):
    d = model_dir(cfg)
    e = Engine(d, tower, [0], dtype, B, mx_sites=mx_sites, lanes=lanes)
    s = torch.cuda.current_stream()
    mc = cfg["model_cfg"]
    E = mc["embed_dim"]
    out = torch.empty((B, E), device="cuda")
    if tower == 0:
        S = mc["vision_cfg"]["image_size"]
        x = torch.randn((B, 3, S, S), device="cuda")
        fn = lambda: e.embed_pixels_device(x.data_ptr(), B, out.data_ptr(), s.cuda_stream)  # noqa: E731
    else:
        T, V = mc["text_cfg"]["context_length"], mc["text_cfg"]["vocab_size"]
        ids = torch.randint(0, V - 2, (B, T), device="cuda", dtype=torch.int64)
        ids[:, -1] = V - 1
        fn = lambda: e.embed_tokens_device(ids.data_ptr(), B, out.data_ptr(), s.cuda_stream)  # noqa: E731
    dt = timed(fn, steps, warmup)
    rate = B / dt
    gf = GFLOP[name.replace("_fp8", "").replace("_full", "")]
    print(json.dumps({"measure": name, "dtype": dtype, "mx_sites": mx_sites if dtype == "fp8" else None,
                      "lanes": e.info()[1],
                      "batch_per_gpu": B, "units_per_s": round(rate, 1),
                      "ms_per_step": round(dt * 1e3, 3), "model_tflops": round(rate * gf / 1e3, 1),
                      "frac_of_2500": round(rate * gf / 1e3 / 2500, 4), "input": "device-resident"}),
          flush=True)
    e.close()


def host_leg(B=256, steps=6, warmup=2):
    d = model_dir(VIT_B_32_CFG)
    e = Engine(d, 0, [0], "bf16", B)
    rng = np.random.default_rng(0)
    u8 = rng.integers(0, 256, (B, 224, 224, 3), dtype=np.uint8)
    mean, std = VIT_B_32_CFG["preprocess_cfg"]["mean"], VIT_B_32_CFG["preprocess_cfg"]["std"]
    px = ((u8.astype(np.float32) / 255 - np.asarray(mean, np.float32)) / np.asarray(std, np.float32))
    px = np.ascontiguousarray(px.transpose(0, 3, 1, 2))
    for kind, fn in (("host_u8", lambda: e.embed_u8(u8, mean, std)), ("host_f32", lambda: e.embed_pixels(px))):
        dt = timed(fn, steps, warmup)
        print(json.dumps({"measure": "b32_vision_" + kind, "batch": B, "units_per_s": round(B / dt, 1),
                          "ms_per_step": round(dt * 1e3, 3),
                          "input": "host buffer (pinned staging + H2D/D2H inside the timing)"}), flush=True)
    e.close()


def captions_leg(B=1024, steps=6, warmup=2):
    """ViT-B/32 text from host token ids at caption lengths (EOT at 8..24, zero padding to
    77): sequence trimming (clipgpu_embed_tokens runs the batch on its first max(EOT)+1
    tokens) on vs off (Engine(trim_text=False)).  Host buffers: H2D/D2H inside the timing."""
    d = model_dir(VIT_B_32_CFG)
    rng = np.random.default_rng(0)
    V = 49408
    ids = np.zeros((B, 77), np.int64)
    ids[:, 0] = V - 2
    eot = rng.integers(8, 25, B)
    for b in range(B):
        ids[b, 1:eot[b]] = rng.integers(1, V - 3, eot[b] - 1)
        ids[b, eot[b]] = V - 1
    res = {}
    for trim in ("1", "0"):
        e = Engine(d, 1, [0], "bf16", B, trim_text=trim == "1")
        dt = timed(lambda: e.embed_tokens(ids), steps, warmup)
        res[trim] = e.embed_tokens(ids)
        print(json.dumps({"measure": "b32_text_captions_" + ("trimmed" if trim == "1" else "full77"), "batch": B,
                          "max_eot": int(eot.max()), "units_per_s": round(B / dt, 1),
                          "ms_per_step": round(dt * 1e3, 3),
                          "input": "host token ids (pinned staging + H2D/D2H inside the timing)"}), flush=True)
        e.close()
    print(json.dumps({"measure": "b32_text_captions_bit_equal", "value": bool(np.array_equal(res["1"], res["0"]))}),
          flush=True)


def photos_leg(B=256, H=480, W=640, steps=4, warmup=1):
    """Decoded 640x480 photos -> embeddings (a3-a7 + forward, BASELINE configs[1] model): the
    reference's CPU resize path restated (host C++ preprocess_batch thread pool + embed_pixels)
    against the GPU crop/resize path (clipgpu_embed_images_rgb8); outputs bit-identical."""
    from open_clip_inference.engine import preprocess_batch_rgb8
    d = model_dir(VIT_B_32_CFG)
    e = Engine(d, 0, [0], "bf16", B)
    rng = np.random.default_rng(1)
    ims = [rng.integers(0, 256, (H, W, 3), dtype=np.uint8) for _ in range(B)]
    pc = VIT_B_32_CFG["preprocess_cfg"]
    legs = (("photos_host_resize", lambda: e.embed_pixels(preprocess_batch_rgb8(ims, 224, "bicubic", "shortest",
                                                                                 pc["mean"], pc["std"]))),
            ("photos_gpu_resize", lambda: e.embed_images_rgb8(ims)))
    for kind, fn in legs:
        dt = timed(fn, steps, warmup)
        print(json.dumps({"measure": "b32_vision_" + kind, "batch": B, "image": f"{W}x{H} RGB8 (bicubic, shortest)",
                          "units_per_s": round(B / dt, 1), "ms_per_step": round(dt * 1e3, 3),
                          "host_threads": min(16, os.cpu_count() or 1)}), flush=True)
    e.close()


def similarity_leg(ni=65536, nt=1000, E=512, steps=5, warmup=2):
    """Facade math on the device: [ni x E] images x [nt x E] labels -> softmax over labels
    (classify for a whole image set), device-resident embeddings; exact-f32 MFMA."""
    import ctypes
    a = torch.nn.functional.normalize(torch.randn(ni, E, device="cuda"), dim=1)
    b = torch.nn.functional.normalize(torch.randn(nt, E, device="cuda"), dim=1)
    out = torch.empty(ni, nt, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    L = _lib.lib()

    def run():
        _lib.check(L.clipgpu_similarity_device(ctypes.c_void_p(a.data_ptr()), ni, ctypes.c_void_p(b.data_ptr()), nt, E,
                                               100.0, 0.0, 0, 1, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s)))
    dt = timed(run, steps, warmup)
    ref = torch.softmax(100.0 * a @ b.T, dim=1)
    err = float((out - ref).abs().max())
    print(json.dumps({"measure": "similarity_softmax", "n_img": ni, "n_txt": nt, "E": E,
                      "ms": round(dt * 1e3, 3), "tflops_f32": round(2 * ni * nt * E / dt / 1e12, 1),
                      "max_abs_err_vs_torch": err}), flush=True)


def latency_leg(steps=50, warmup=10):
    """Single-item latency (the reference's embed_image / embed_text calls, B = 1) through the
    host entry points: pinned staging + H2D + forward + D2H + synchronise, ViT-B/32."""
    d = model_dir(VIT_B_32_CFG)
    mean, std = VIT_B_32_CFG["preprocess_cfg"]["mean"], VIT_B_32_CFG["preprocess_cfg"]["std"]
    ve = Engine(d, 0, [0], "bf16", 8)
    te = Engine(d, 1, [0], "bf16", 8)
    rng = np.random.default_rng(3)
    u8 = rng.integers(0, 256, (1, 224, 224, 3), dtype=np.uint8)
    px = np.ascontiguousarray(((u8.astype(np.float32) / 255 - np.asarray(mean, np.float32)) /
                               np.asarray(std, np.float32)).transpose(0, 3, 1, 2))
    ids = np.zeros((1, 77), np.int64)
    ids[0, :5] = [49406, 320, 1125, 539, 49407]
    photo = [rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)]
    for name, fn in (("b32_embed_image_f32", lambda: ve.embed_pixels(px)),
                     ("b32_embed_image_photo_gpu_resize", lambda: ve.embed_images_rgb8(photo)),
                     ("b32_embed_text", lambda: te.embed_tokens(ids))):
        for _ in range(warmup):
            fn()
        ts = []
        for _ in range(steps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        print(json.dumps({"measure": "latency_" + name, "batch": 1, "p50_ms": round(ts[len(ts) // 2] * 1e3, 3),
                          "p90_ms": round(ts[int(len(ts) * 0.9)] * 1e3, 3)}), flush=True)
    ve.close()
    te.close()


if __name__ == "__main__":
    which = sys.argv[1:] or ["host", "photos", "similarity", "latency", "so400m", "h14"]
    if "host" in which:
        host_leg()
    if "captions" in which:
        captions_leg()
    if "photos" in which:
        photos_leg()
    if "similarity" in which:
        similarity_leg()
    if "latency" in which:
        latency_leg()
    if "so400m" in which:
        device_leg("so400m_vision", SO400M_16_SIGLIP2_384_CFG, 0, 128)
    if "h14" in which:
        device_leg("h14_vision", VIT_H_14_378_CFG, 0, 64)
        device_leg("h14_text", VIT_H_14_378_CFG, 1, 64)
    if "h14fp8" in which:
        # configs[4]'s fp8 MFMA weight path at the north-star tolerance: vision with
        # QKV in MX-fp8 (cos >= 0.9999), text in bf16 -- no MX text split meets the bar at any
        # speed gain (per-site and per-layer sweeps, profiles/r04_mx_layer_*.jsonl)
        device_leg("h14_vision_fp8", VIT_H_14_378_CFG, 0, 64, dtype="fp8", mx_sites="qkv")
        device_leg("h14_text", VIT_H_14_378_CFG, 1, 64)
    if "h14fp8full" in which:  # the full MX split (QKV, c_fc, c_proj): throughput mode, below the bar
        device_leg("h14_vision_fp8_full", VIT_H_14_378_CFG, 0, 64, dtype="fp8")
        device_leg("h14_text_fp8_full", VIT_H_14_378_CFG, 1, 64, dtype="fp8")
    if "lanesab" in which:  # one vs two device lanes at the large-model shards (table tiles), interleaved
        for rnd in range(2):
            for lanes in (1, 2):
                device_leg("so400m_vision", SO400M_16_SIGLIP2_384_CFG, 0, 128, lanes=lanes)
                device_leg("h14_vision", VIT_H_14_378_CFG, 0, 64, lanes=lanes)
                device_leg("h14_text", VIT_H_14_378_CFG, 1, 64, lanes=lanes)
    if "so400mtext" in which:  # the SigLIP2 text tower of the configs[3] model folder
        device_leg("so400m_text", SO400M_16_SIGLIP2_384_CFG, 1, 128)
    if "so400mfp8" in which:
        device_leg("so400m_vision_fp8", SO400M_16_SIGLIP2_384_CFG, 0, 128, dtype="fp8")
    if "b32fp8" in which:
        device_leg("b32_vision_fp8", VIT_B_32_CFG, 0, 256, dtype="fp8")
