#!/usr/bin/env python3
"""clipgpu benchmark — BASELINE.json metric:
"images/sec + texts/sec embedding, ViT-B/32-224, batch 256, 1/2/4/8 MI355X".

One step = one pass of the hot path over one batch of synthetic input resident in
HBM: ViT-B/32-224 vision tower on 256 normalised f32 images per GPU
(BASELINE.json configs[1]) -> L2-normalised [256, 512], then (N > 1) the RCCL
all-gather of the embedding matrix over xGMI (weak scaling).
Weights are seeded synthetic (no checkpoint can be fetched); arithmetic in bf16
with f32 accumulation / residual adds / LayerNorm statistics / softmax; the residual
stream stored in f16 (the library default for bf16 engines; `--residual f32` for f32).

Also reported: texts/s for configs[2] (text tower, batch 1024 x 77 tokens);
roofline of the dominant kernel (the trunk GEMM site with the most time per step) from HIP
events on the launch stream;
end-to-end legs through the host-buffer entry points (PCIe included; N = 1);
CPU baseline = the fp32 torch CPU port of the same graphs (oracle/torch_cpu.py) on a bounded
sample of the same inputs on rank 0, which also checks the GPU rows (cosine).

Launch: python bench.py [--gpus N --steps K --warmup W].  N > 1: one rank per GPU.  Started without a
torch.distributed launcher (no WORLD_SIZE in the environment), bench.py starts the N ranks itself --
`python -m torch.distributed.run --nproc-per-node N` as a child process, before anything touches the GPU
-- and exits with its status; rank 0 prints the JSON line.  Under a launcher, WORLD_SIZE must equal
--gpus (a mismatch exits with status 2), so `n_gpus` is always --gpus.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import torch  # noqa: E402  (import torch before the native lib: one HIP runtime per process)
import torch.distributed as dist
import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))

from open_clip_inference import _lib  # noqa: E402
from open_clip_inference.engine import Engine, profile_enable, profile_read  # noqa: E402
from open_clip_inference.parallel import init_engine_comm  # noqa: E402

# ViT-B/32 (open_clip timm/vit_base_patch32_clip_224.openai)
CFG = {
    "model_cfg": {"embed_dim": 512, "quick_gelu": True,
                  "vision_cfg": {"image_size": 224, "layers": 12, "width": 768, "patch_size": 32},
                  "text_cfg": {"context_length": 77, "vocab_size": 49408, "width": 512, "heads": 8,
                               "layers": 12}},
    "preprocess_cfg": {"mean": [0.48145466, 0.4578275, 0.40821073],
                       "std": [0.26862954, 0.26130258, 0.27577711]},
}
MODEL_CONFIG = {"logit_scale": 100.0, "logit_bias": 0.0, "activation_function": "softmax",
                "tokenizer_needs_lowercase": False, "pad_id": 0, "vocab_size": 49408}

# Algorithmic work per unit: 2 x MAC over all matmuls.
# The engine prunes the last layer to the pooled token after attention (engine.hip trunk,
# clipgpu_options.prune_last, bit-identical embeddings): `executed` counts the MFMA work that runs.
PRUNE_LAST = True  # the engine default (clipgpu_options.prune_last)


def vit_flops(B, executed=False):
    S, P, D, L, M, E = 224, 32, 768, 12, 3072, 512
    g2 = (S // P) ** 2
    N = g2 + 1
    patch = 2 * B * g2 * D * 3 * P * P
    per_layer = 2 * B * N * (3 * D * D + D * D + 2 * D * M) + 2 * 2 * B * N * N * D
    pruned = 2 * B * (N - 1) * (D * D + 2 * D * M) if executed and PRUNE_LAST else 0
    return patch + L * per_layer + 2 * B * D * E - pruned


def text_flops(B, T=77, executed=False):
    D, L, M, E = 512, 12, 2048, 512
    pruned = 2 * B * (T - 1) * (D * D + 2 * D * M) if executed and PRUNE_LAST else 0
    return L * (2 * B * T * (3 * D * D + D * D + 2 * D * M) + 2 * 2 * B * T * T * D) + 2 * B * D * E - pruned


# GemmTile ids the library builds (csrc/kernels/kernels.hpp kGemmTiles)
# trunk GEMM sites of the ViT-B/32 vision tower: (N, K), and what the epilogue adds
SITE_SHAPES = {"qkv": (2304, 768), "out_proj": (768, 768), "c_fc": (3072, 768), "c_proj": (768, 3072)}
SITE_EPI = {"qkv": "{ln}+bias", "out_proj": "+bias, {x} residual", "c_fc": "{ln}+QuickGELU",
            "c_proj": "+bias, {x} residual"}
TILE_NAMES = {0: "heuristic", 2: "256x128", 3: "256x256", 13: "192x256w8", 14: "256x256rs",
              15: "160x128rs", 17: "160x128w8rs", 18: "256x256half", 26: "224x192w8", 100: "skinny", 101: "general"}
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
B_VISION = 256
B_TEXT = 1024


def make_model_dir():
    d = tempfile.mkdtemp(prefix="clipgpu_bench_")
    for name, obj in (("open_clip_config.json", CFG), ("model_config.json", MODEL_CONFIG),
                      ("clipgpu_synthetic.json", {"seed": 1234})):
        with open(os.path.join(d, name), "w") as f:
            json.dump(obj, f)
    return d


def synth_inputs(rank, device):
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    u8 = torch.randint(0, 256, (B_VISION, 224, 224, 3), dtype=torch.uint8, generator=g)
    mean = torch.tensor(CFG["preprocess_cfg"]["mean"], dtype=torch.float32)
    std = torch.tensor(CFG["preprocess_cfg"]["std"], dtype=torch.float32)
    px = ((u8.float() / 255.0 - mean) / std).permute(0, 3, 1, 2).contiguous()
    ids = torch.randint(0, 49406, (B_TEXT, 77), dtype=torch.int64, generator=g)
    ids[:, 0] = 49406
    ids[:, 76] = 49407
    return px.to(device), ids.to(device)


def num_cpus_rule():
    """num_cpus::get(): the reference's ONNX Runtime intra-op thread count (src/onnx.rs:18-22,
    `intra_threads = num_cpus::get()`).  num_cpus 1.x on Linux returns the CPUs in the process's
    scheduler affinity, capped by a cgroup CPU quota when one is set (cgroup v2 cpu.max, v1
    cpu.cfs_quota_us / cpu.cfs_period_us; quota / period rounded up)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = -(-int(q) // int(per))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0 and per > 0:
                quota = -(-q // per)
        except (OSError, ValueError):
            pass
    return max(1, min(n, quota) if quota else n), quota


def host_info():
    """Host cores as the CPU leg sees them (the GPU box's CPU share, not the machine's count)."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    rule, quota = num_cpus_rule()
    return {"nproc_affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count(), "cpu_model": model,
            "cgroup_cpu_quota": quota, "num_cpus_rule": rule,
            "torch_threads": torch.get_num_threads(), "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(px_host, ids_host, gpu_vision, gpu_text, fp8_vision=None, target_s=12.0):
    """The CPU leg (rank 0, N = 1): the reference's graphs in fp32 on torch's CPU kernels
    (oracle/torch_cpu.py -- the closest buildable proxy of the reference's ONNX Runtime CPU path,
    src/onnx.rs:18-22), all host threads torch has, on the bench's own inputs: a bounded sample
    of the vision batch and of the text batch.  Its embeddings also check the GPU rows of the
    same inputs (cosine), which ties the timed numbers to a correctness check."""
    from oracle import torch_cpu, weights
    from oracle.model_spec import text_spec_from_cfg, vision_spec_from_cfg
    v = vision_spec_from_cfg(CFG["model_cfg"])
    t = text_spec_from_cfg(CFG["model_cfg"])
    vm = torch_cpu.VisionCPU(weights.vision_weights(v, 1234), v)
    tm = torch_cpu.TextCPU(weights.text_weights(t, 1234), t)

    def run(model, data, budget, chunk):
        model(data[:2])  # warm
        t0 = time.perf_counter()
        model(data[:chunk])
        per = (time.perf_counter() - t0) / chunk
        n = int(min(len(data), max(chunk, budget / max(per, 1e-9)))) // chunk * chunk
        outs = []
        t0 = time.perf_counter()
        for i in range(0, n, chunk):
            outs.append(model(data[i:i + chunk]))
        return np.concatenate(outs), time.perf_counter() - t0

    def cos_min(a, b):
        a = np.asarray(a, np.float64)
        b = np.asarray(b, np.float64)
        return float(((a * b).sum(1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))).min())

    # Threads: the reference's rule (num_cpus::get(), src/onnx.rs:18-22), held to the CPU share the
    # GPU pool grants this box (OMP_NUM_THREADS, set by the pool: a box's worker pools must not
    # exceed it) when that is smaller -- both numbers are reported in `host`.
    rule, _ = num_cpus_rule()
    share = int(os.environ.get("OMP_NUM_THREADS") or rule)
    prev = torch.get_num_threads()
    torch.set_num_threads(max(1, min(rule, share)))
    ve, vdt = run(vm, px_host, target_s, 32)
    te, tdt = run(tm, ids_host, target_s, 128)
    cores = torch.get_num_threads()
    torch.set_num_threads(prev)
    res = {"value": round(len(ve) / vdt, 2), "unit": "images/s", "cores": cores, "kind": "port",
           "sample": f"{len(ve)} of the bench's 256 synthetic 224x224 images (batches of 32), ViT-B/32 vision tower, "
                     f"fp32 torch CPU port of the graph (oracle/torch_cpu.py), {cores} threads, {vdt:.1f} s",
           "host": host_info(),
           "text": {"value": round(len(te) / tdt, 2), "unit": "texts/s",
                    "sample": f"{len(te)} of the bench's 1024 x 77-token sequences (batches of 128), {tdt:.1f} s"},
           "gpu_vs_cpu_cos_min": {"vision_bf16": cos_min(gpu_vision[:len(ve)], ve),
                                  "text_bf16": cos_min(gpu_text[:len(te)], te) if gpu_text is not None else None}}
    if fp8_vision is not None:
        res["gpu_vs_cpu_cos_min"]["vision_fp8"] = cos_min(fp8_vision[:len(ve)], ve)
    return res


def load_traffic(site, rows_per_launch, tiles, form):
    """HBM bytes per launch of the roofline kernel: NOT measured in this run -- read from the
    committed PMC summary (separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench,
    gfx950 FETCH_SIZE x2 correction, tools/pmc_traffic.py); its `source` names the run it came from.
    Only used when it was measured for this site at this run's rows per launch AND with this run's
    GEMM tiles (the record's `tiles`) and epilogue form (`form`: "f16 residual" / "f32 residual" for
    out_proj / c_proj, "LayerNorm folded" or "" for c_fc, matched against the record's `kernel` text);
    otherwise null, with the reason in traffic_source."""
    p = os.path.join(ROOT, "profiles", "pmc_c_fc.json")
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        key = f"{site}:{int(rows_per_launch)}"
        rec = d.get("by_site_rows", {}).get(key)
        if rec is None and site == "c_fc":
            rec = d.get("by_rows", {}).get(str(int(rows_per_launch)))
        if rec is None:
            return None, (f"profiles/pmc_c_fc.json has no {site} measurement at {int(rows_per_launch)} rows per "
                          f"launch (has {sorted(d.get('by_site_rows', {}))})")
        if rec.get("tiles") != tiles:
            return None, (f"profiles/pmc_c_fc.json's record at {int(rows_per_launch)} rows was taken with tiles "
                          f"{rec.get('tiles')}, this run uses {tiles}: not applicable")
        k = rec.get("kernel", "")
        if (form and form not in k) or (not form and "LayerNorm folded" in k):
            return None, (f"profiles/pmc_c_fc.json's {site} record ({k}) is not this run's epilogue form "
                          f"({form or 'no LayerNorm fold'}): not applicable")
        return rec.get("hbm_bytes_per_launch"), "profiles/pmc_c_fc.json: " + rec.get("source", "rocprofv3 PMC passes")
    return None, None


def measure_windows(step, engine, n, steps, dt_first, dev):
    """Repeated windows after the timed one (N = 1), so a few-% change can be told from box-to-box
    and run-to-run spread.  Each window is `steps` forward steps timed like `value`; windows
    alternate:
    - plain (`images_s`), followed at once by a 2 ms one-wave clock probe (clipgpu_test_clock_probe:
      s_memtime ticks over s_memrealtime's 100 MHz): the clock as the load ends (`sclk_after_mhz`);
      some boxes boost back within that time, so it is not the clock under load;
    - probed (`images_s_probed`): the same probe on a side stream for 60 % of the first window's
      wall time, beside the forward, reads the shader clock the chip holds under the forward's load
      (`sclk_mhz`; MI355X_MICROARCH.md, DVFS give-back).  The probe's wave keeps one CU from hosting
      a one-block-per-CU GEMM block, so these windows run a few % slower.
    Then profiled windows give the mean c_fc launch time (HIP events at the kernel boundaries,
    lanes serialized, no graphs), each with the probe beside it."""
    import statistics
    L = _lib.lib()
    side = torch.cuda.Stream(dev)
    probe = torch.zeros(2, dtype=torch.int64, device=dev)
    probe_us = max(1000, int(0.6 * dt_first * 1e6))

    def mhz():
        t = probe.cpu().tolist()
        return 100.0 * t[0] / t[1] if t[1] > 0 else None

    def window(fn, beside):
        torch.cuda.synchronize()
        if beside:
            _lib.check(L.clipgpu_test_clock_probe(ctypes.c_void_p(side.cuda_stream), probe_us,
                                                  ctypes.c_void_p(probe.data_ptr())))
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if beside:
            return wall, mhz(), out
        _lib.check(L.clipgpu_test_clock_probe(None, 2000, ctypes.c_void_p(probe.data_ptr())))
        return wall, mhz(), out

    def run_steps():
        for _ in range(steps):
            step()

    rates, after, rates_probe, clocks = [], [], [], []
    for _ in range(n):
        wall, m, _ = window(run_steps, False)
        rates.append(B_VISION * steps / wall)
        after.append(m)
        wall, m, _ = window(run_steps, True)
        rates_probe.append(B_VISION * steps / wall)
        clocks.append(m)
    fc_us, fc_clk = [], []
    for _ in range(max(1, min(n, 3))):
        profile_enable(engine, ["c_fc"])

        def prof_steps():
            run_steps()
            return profile_read(engine, "c_fc")
        _, m, (ms, cnt) = window(prof_steps, True)
        profile_enable(engine, [])
        fc_us.append(1e3 * ms / max(cnt, 1))
        fc_clk.append(m)
    good = [c for c in clocks if c]
    med = lambda xs: round(statistics.median([x for x in xs if x]), 1) if any(xs) else None  # noqa: E731
    r1 = lambda xs: [round(x, 1) if x else None for x in xs]  # noqa: E731
    return {"n": n, "steps": steps,
            "images_s": r1(rates),
            "min": round(min(rates), 1), "median": round(statistics.median(rates), 1), "max": round(max(rates), 1),
            "sclk_mhz": r1(clocks), "sclk_mhz_median": med(clocks),
            "sclk_after_mhz": r1(after), "sclk_after_mhz_median": med(after),
            "images_s_probed": r1(rates_probe),
            "images_s_per_ghz_median": round(statistics.median(r / (c / 1e3) for r, c in zip(rates_probe, clocks) if c), 1)
            if good else None,
            "c_fc_us": [round(u, 2) for u in fc_us], "c_fc_sclk_mhz": r1(fc_clk),
            "note": "windows after the timed one (same steps each), alternating plain (images_s; then a 2 ms probe: "
                    "sclk_after_mhz, the clock as the load ends) and clock-probed (images_s_probed: a one-wave "
                    "s_memtime / s_memrealtime probe on a side stream beside the forward: sclk_mhz, the clock under "
                    "load); c_fc from profiled windows (lanes serialized)"}


def _timed_calls(call, steps):
    """(median, mean) seconds per call over `steps` calls after one warm call: the end-to-end legs
    report the median, so one scheduling hiccup on the host does not set a leg's number."""
    call()
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        call()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), float(np.mean(ts))


def host_leg(engine, kind, host, steps, registered=False):
    """Host-buffer throughput through the C ABI (H2D + forward + D2H, PCIe included), units per
    second over `steps` calls after one warm call.  Pageable arrays go through the engine's pinned
    staging; `registered` pins the caller's input and output arrays first (clipgpu_host_register:
    direct DMA).  Either way the engine moves the batch in even per-lane chunks (engine.hip
    host_chunks), each chunk's forward starting once its H2D has landed."""
    from open_clip_inference.engine import host_buffer, host_register, host_unregister
    if registered:  # page-owning arrays (registration pins whole pages)
        buf = host_buffer(host.shape, host.dtype)
        buf[...] = host
        host = buf
        out = host_buffer((len(host), engine.embed_dim), np.float32)
    else:
        host = np.ascontiguousarray(host)
        out = np.empty((len(host), engine.embed_dim), np.float32)
    call = {"u8": lambda: engine.embed_u8(host, CFG["preprocess_cfg"]["mean"], CFG["preprocess_cfg"]["std"], out=out),
            "f32": lambda: engine.embed_pixels(host, out=out),
            "tokens": lambda: engine.embed_tokens(host, out=out)}[kind]
    if registered:
        host_register(host)
        host_register(out)
    try:
        med, mean = _timed_calls(call, steps)
    finally:
        if registered:
            host_unregister(host)
            host_unregister(out)
    shape = ",".join(str(d) for d in host.shape)
    entry = {"u8": f"clipgpu_embed_u8 (u8 NHWC [{shape}])", "f32": f"clipgpu_embed_pixels (f32 NCHW [{shape}])",
             "tokens": f"clipgpu_embed_tokens (i64 ids [{shape}], full-length rows: no trimming)"}[kind]
    return {"value": round(len(host) / med, 1), "unit": "texts/s" if kind == "tokens" else "images/s",
            "ms_per_call": round(med * 1e3, 3), "ms_per_call_mean": round(mean * 1e3, 3), "calls": steps,
            "entry": entry,
            "buffers": "caller-registered (direct DMA)" if registered else "pageable (pinned staging)"}


def images_leg(engine, images, steps, host_preprocess=False):
    """The drop-in entry point of embed_images(&[DynamicImage]) (src/vision.rs:100-162: preprocess_batch
    + session.run): decoded RGB8 images of any size in, embeddings out.  GPU path:
    clipgpu_embed_images_rgb8 (crop / resize / normalise on the GPU, bit-identical to the host
    preprocessing); host path: clipgpu_preprocess_batch (the host thread pool) + clipgpu_embed_pixels."""
    from open_clip_inference.engine import preprocess_batch_rgb8
    pc = CFG["preprocess_cfg"]

    # The GPU path is timed at the C ABI with its arguments marshalled once (a Rust caller passes its
    # images' pointers and sizes straight through); the Python wrapper's per-call marshalling of 256
    # arrays is reported beside it.
    n = len(images)
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in images])
    ws = (ctypes.c_int * n)(*[a.shape[1] for a in images])
    hs = (ctypes.c_int * n)(*[a.shape[0] for a in images])
    out = np.empty((n, engine.embed_dim), np.float32)
    L = _lib.lib()

    def call():
        if host_preprocess:
            px = preprocess_batch_rgb8(images, 224, "bicubic", "shortest", pc["mean"], pc["std"])
            return engine.embed_pixels(px)
        _lib.check(L.clipgpu_embed_images_rgb8(engine.handle, ptrs, ws, hs, n, out.ctypes.data))
    med, mean = _timed_calls(call, steps)
    extra = {}
    if not host_preprocess:
        wmed, _ = _timed_calls(lambda: engine.embed_images_rgb8(images), steps)
        extra = {"python_wrapper_ms_per_call": round(wmed * 1e3, 3)}
    h, w = images[0].shape[:2]
    return {"value": round(len(images) / med, 1), "unit": "images/s", "ms_per_call": round(med * 1e3, 3),
            "ms_per_call_mean": round(mean * 1e3, 3), "calls": steps, **extra,
            "entry": ("clipgpu_preprocess_batch (host, bicubic shortest-side resize + centre crop + normalise) + "
                      "clipgpu_embed_pixels" if host_preprocess else
                      "clipgpu_embed_images_rgb8 (resize + centre crop + normalise on the GPU)") +
                     f": {len(images)} decoded {w}x{h} RGB8 images per call"}


def free_port():
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(n, argv):
    """--gpus N > 1 without a launcher: N rank processes through torch.distributed.run (a child process:
    this process has not touched the GPU and never execs), one per GPU, rendezvous on 127.0.0.1.  Their
    output passes through; returns the launcher's exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def resolve_world(gpus, env):
    """(world, rank, local rank) of this process, or an int exit status for main() to return: launch
    the ranks (no WORLD_SIZE and gpus > 1) or refuse a WORLD_SIZE that is not --gpus."""
    if gpus < 1:
        print(f"bench.py: --gpus {gpus} < 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in env:
        if gpus > 1:
            return ("launch", gpus)
        return 1, 0, 0
    world = int(env["WORLD_SIZE"])
    if world != gpus:
        print(f"bench.py: --gpus {gpus} but WORLD_SIZE={world} (the launcher started {world} ranks): refusing "
              f"to report n_gpus={world} for a {gpus}-GPU request", file=sys.stderr)
        return 2
    return world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))


def plumbing_check(world, rank):
    """--plumbing-check: the N > 1 rank plumbing without a GPU call (tests/test_cpu_bench_launcher.py):
    the gloo control plane the bench uses, a barrier and a gather of (rank, local rank, world) from
    every rank; rank 0 prints them as one JSON line."""
    dist.init_process_group("gloo")
    me = torch.tensor([rank, int(os.environ.get("LOCAL_RANK", "0")), world], dtype=torch.int64)
    got = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(got, me)
    dist.barrier()
    if rank == 0:
        print(json.dumps({"plumbing": [g.tolist() for g in got], "n_gpus": world}), flush=True)
    dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-text", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "fp8"])
    ap.add_argument("--no-fp8", action="store_true", help="skip the fp8 side measurement")
    ap.add_argument("--breakdown", action="store_true", help="per-kernel-class ms per step (serialized lanes)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) legs")
    ap.add_argument("--tiles", default="",
                    help="vision engine: pin the GEMM tiles q,o,f,p (clipgpu_options.gemm_tiles; PMC passes and "
                         "A/B runs pin the un-profiled bench's tiles); the patch GEMM takes p's")
    ap.add_argument("--lanes", type=int, default=0, help="vision engine: pin the device lanes (0 = the table's)")
    ap.add_argument("--text-tiles", default="", help="text engine: pin the GEMM tiles q,o,f,p (A/B runs)")
    ap.add_argument("--text-lanes", type=int, default=0, help="text engine: pin the device lanes (0 = the table's)")
    ap.add_argument("--windows", type=int, default=5,
                    help="N = 1: repeated K-step windows after the timed one (min / median / max images/s, the "
                         "shader clock of each window, and the c_fc launch time per window); 0 skips them")
    ap.add_argument("--ln-fold", default=None, choices=["on", "off"],
                    help="ln_1 / ln_2 folded into the QKV / c_fc GEMMs (clipgpu_options.ln_fold; default: the library's)")
    ap.add_argument("--residual", default=None, choices=["f32", "f16"],
                    help="the residual stream's storage (clipgpu_options.residual; default: the library's)")
    ap.add_argument("--gather", action="store_true",
                    help="N = 1: run the data-parallel path anyway (gloo control plane, the engine's RCCL "
                         "communicator, gathered entry points) -- a one-GPU rehearsal of N > 1")
    ap.add_argument("--plumbing-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    w = resolve_world(args.gpus, os.environ)
    if isinstance(w, int):
        return w
    if w[0] == "launch":
        return launch_ranks(w[1], sys.argv[1:])
    world, rank, local = w
    if args.plumbing_check:
        return plumbing_check(world, rank) if world > 1 else 0
    # dp: the data-parallel path (every N > 1 run; --gather rehearses it at N = 1 on one GPU)
    dp = world > 1 or args.gather
    if world > 1:
        # control plane only (barriers, max-over-ranks timing, the RCCL unique id); the data path's
        # collective is the engine's own RCCL communicator (clipgpu_comm_init_rank)
        dist.init_process_group("gloo")
    elif dp:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    mdir = make_model_dir()
    fold = {None: None, "on": True, "off": False}[args.ln_fold]
    vopts = {"lanes": args.lanes, "residual": args.residual, "ln_fold": fold}
    if args.tiles:
        pins = [int(t) for t in args.tiles.split(",")]
        vopts.update(gemm_tiles=pins, patch_tile=pins[3])
    ve = Engine(mdir, _lib.TOWER_VISION, [local], args.dtype, B_VISION, **vopts)
    if dp:
        init_engine_comm(ve)
    px, ids = synth_inputs(rank, dev)
    out_full = torch.empty((world * B_VISION, 512), device=dev, dtype=torch.float32)
    out = out_full[rank * B_VISION:(rank + 1) * B_VISION]  # this rank's rows
    stream = torch.cuda.current_stream(dev)

    def vision_step():
        if dp:  # forward of this rank's 256 rows + one RCCL all-gather of [world*256, 512]
            ve.embed_pixels_gather_device([px.data_ptr()], [B_VISION] * world, [out_full.data_ptr()],
                                          [stream.cuda_stream])
        else:
            ve.embed_pixels_device(px.data_ptr(), B_VISION, out.data_ptr(), stream.cuda_stream)

    def timed(step, steps, warmup, prof_engine=None, prof_cats=None, concurrent=False):
        for _ in range(warmup):
            step()
        if prof_engine is not None:
            profile_enable(prof_engine, list(prof_cats), concurrent=concurrent)
        if dp:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        if dp:
            dist.barrier()
        dt = time.perf_counter() - t0
        if dp:
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        prof = None
        if prof_engine is not None:
            prof = {c: profile_read(prof_engine, c) for c in prof_cats}
            profile_enable(prof_engine, [])
        return dt, prof

    tiles = (ctypes.c_int * 4)()
    _lib.check(_lib.lib().clipgpu_test_engine_tiles(ve._h, tiles))
    dev_lanes = ctypes.c_int()
    _lib.check(_lib.lib().clipgpu_test_engine_lanes(ve._h, ctypes.byref(dev_lanes)))
    x_store, ln_fold = ctypes.c_int(), ctypes.c_int()
    _lib.check(_lib.lib().clipgpu_test_engine_residual(ve._h, ctypes.byref(x_store), ctypes.byref(ln_fold)))
    x_store = "f16" if x_store.value == 2 else "f32"  # CLIPGPU_RESIDUAL_F16 / _F32
    ln_fold = bool(ln_fold.value)
    mx_names = {0: "heuristic", 2: "mx256x128", 3: "mx128x128"}  # fp8 engines: QKV / c_fc / c_proj sites
    fp8 = args.dtype == "fp8"
    gemm_tiles = {site: (mx_names if fp8 and site != "out_proj" else TILE_NAMES).get(t, f"tile{t}")
                  for site, t in zip(["qkv", "out_proj", "c_fc", "c_proj"], tiles)}
    # the dominant kernel's peak: the dense bf16 MFMA rate, or the block-scaled MX-fp8 rate (2x)
    peak = PEAK_BF16_TFLOPS * (2 if fp8 else 1)

    dt, _ = timed(vision_step, args.steps, args.warmup)
    images = world * B_VISION * args.steps
    value = images / dt
    ms_per_step = dt * 1e3 / args.steps
    # Per-launch kernel time of the four trunk GEMM sites: a separate pass with HIP events at the
    # kernel boundaries of every launch.  Profiling runs the engine's two lanes (half-batch
    # sub-forwards) one after the other instead of concurrently, so it is kept out of the timed
    # loop; launch shapes are the same.
    psteps = max(3, args.steps // 2)
    _, site_prof = timed(vision_step, psteps, 1, ve, SITE_SHAPES)
    fc_ms, fc_n = site_prof["c_fc"]
    # The same launches timed in the timed step's regime: both lanes running (CLIPGPU_PROFILE_CONCURRENT:
    # no serialization, no graph replay), each GEMM's event pair at its own kernel boundaries.
    _, site_prof_cc = timed(vision_step, psteps, 1, ve, SITE_SHAPES, concurrent=True)
    windows = None
    if world == 1 and args.windows > 0:
        windows = measure_windows(vision_step, ve, args.windows, args.steps, dt, dev)

    # Per-site figures (M = rows per launch; the counts are the full-row launches: 12 layers, or 11
    # when the last one is pruned to the pooled rows and profiled as "last_layer", x lanes per
    # step).  The roofline kernel is the dominant one: the site with the most GEMM time per step.
    fc_layers = 11 if PRUNE_LAST else 12
    sites = {}
    for site, (N, K) in SITE_SHAPES.items():
        ms, n = site_prof[site]
        # qkv runs on every token in every layer (the pruned last layer's attention needs all keys)
        rows = B_VISION * 50 * (12 if site == "qkv" else fc_layers) * psteps / max(n, 1)
        avg_s = (ms / 1e3) / max(n, 1)
        tf = 2.0 * rows * N * K / avg_s / 1e12 if n else 0.0
        # blocks per launch (the launcher's persistent grid) and the CU-time view: a launch holds
        # min(blocks, CUs) CUs for its duration beside the other lane; cu_frac = FLOPs / (that CU time x
        # the per-CU peak), i.e. frac x CUs / min(CUs, blocks) on the concurrent duration
        grid = ctypes.c_int()
        _lib.check(_lib.lib().clipgpu_test_gemm_grid(int(tiles[list(SITE_SHAPES).index(site)]), int(rows), N, K,
                                                     ctypes.byref(grid)))
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        held = min(grid.value, cus)
        ms_cc, n_cc = site_prof_cc[site]
        avg_cc = (ms_cc / 1e3) / max(n_cc, 1)
        tf_cc = 2.0 * rows * N * K / avg_cc / 1e12 if n_cc else 0.0
        sites[site] = {"shape": f"{int(rows)}x{N}x{K}", "rows_per_launch": int(rows), "tile": gemm_tiles[site],
                       "avg_launch_us": round(avg_s * 1e6, 2), "us_per_step": round(ms * 1e3 / psteps, 1),
                       "tflops": round(tf, 1), "frac": round(tf / peak, 4),
                       "blocks": grid.value, "cus_held": held,
                       "concurrent": {"avg_launch_us": round(avg_cc * 1e6, 2), "tflops": round(tf_cc, 1),
                                      "frac": round(tf_cc / peak, 4),
                                      "cu_us_per_step": round(ms_cc * 1e3 / psteps * held / cus, 1),
                                      "cu_frac": round(tf_cc / peak * cus / held, 4)}}
    dom = max(sites, key=lambda k: sites[k]["us_per_step"])
    dom_epi = SITE_EPI[dom].format(x=x_store, ln="LayerNorm folded, " if ln_fold else "")
    fc_rows_per_launch = sites["c_fc"]["rows_per_launch"]
    whole_tflops = vit_flops(B_VISION, executed=True) * args.steps / dt / 1e12 / 1.0

    # Per-kernel-class time per step (lanes serialized, no graph): where the step goes.
    breakdown = None
    if args.breakdown:
        from open_clip_inference.engine import PROFILE_CATEGORIES
        bsteps = max(3, args.steps // 2)
        for _ in range(2):
            vision_step()
        profile_enable(ve, PROFILE_CATEGORIES)
        torch.cuda.synchronize()
        for _ in range(bsteps):
            vision_step()
        torch.cuda.synchronize()
        breakdown = {}
        for c in PROFILE_CATEGORIES:
            ms, n = profile_read(ve, c)
            if n:
                breakdown[c] = {"ms_per_step": round(ms / bsteps, 4), "launches_per_step": n // bsteps}
        profile_enable(ve, [])

    # The fp8 (MX) engine of the same workload beside the bf16 value (BASELINE configs[4]'s
    # weight path on the bench model): throughput and the cosine of its embeddings to the
    # bf16 engine's on the same input (the fp8 path is lossy).  Not `value`.
    fp8_info = None
    fout_host = None
    if world == 1 and not fp8 and not args.no_fp8:
        fe = Engine(mdir, _lib.TOWER_VISION, [local], "fp8", B_VISION)
        fout = torch.empty_like(out)

        def fp8_step():
            fe.embed_pixels_device(px.data_ptr(), B_VISION, fout.data_ptr(), stream.cuda_stream)
        fdt, _ = timed(fp8_step, args.steps, args.warmup)
        vision_step()
        torch.cuda.synchronize()
        cos = torch.nn.functional.cosine_similarity(fout, out, dim=1)
        fout_host = fout.cpu().numpy()
        f_tflops = vit_flops(B_VISION, executed=True) * args.steps / fdt / 1e12
        fp8_info = {"value": round(B_VISION * args.steps / fdt, 1), "unit": "images/s",
                    "ms_per_step": round(fdt * 1e3 / args.steps, 3),
                    "whole_forward_tflops": round(f_tflops, 1),
                    "frac_of_mx_fp8_peak": round(f_tflops / (2 * PEAK_BF16_TFLOPS), 4),
                    "cos_vs_bf16_min": round(float(cos.min()), 6), "cos_vs_bf16_mean": round(float(cos.mean()), 6),
                    "note": "MX-fp8 QKV/c_fc/c_proj (e4m3 + E8M0 per 32, v_mfma_scale_f32_32x32x64_f8f6f4); "
                            "frac against the 5 PF block-scaled MX peak (the mix also runs bf16 GEMMs); "
                            "cosine vs the fp32 CPU port in cpu_baseline.gpu_vs_cpu_cos_min.vision_fp8"}
        fe.close()

    text = None
    tout_host = None
    if not args.no_text:
        topts = {"lanes": args.text_lanes, "residual": args.residual, "ln_fold": fold}
        if args.text_tiles:
            topts["gemm_tiles"] = [int(t) for t in args.text_tiles.split(",")]
        te = Engine(mdir, _lib.TOWER_TEXT, [local], args.dtype, B_TEXT, **topts)
        if dp:
            init_engine_comm(te)
        tout_full = torch.empty((world * B_TEXT, 512), device=dev, dtype=torch.float32)
        tout = tout_full[rank * B_TEXT:(rank + 1) * B_TEXT]

        def text_step():
            if dp:
                te.embed_tokens_gather_device([ids.data_ptr()], [B_TEXT] * world, [tout_full.data_ptr()],
                                              [stream.cuda_stream])
            else:
                te.embed_tokens_device(ids.data_ptr(), B_TEXT, tout.data_ptr(), stream.cuda_stream)

        tsteps = max(3, args.steps // 2)
        tdt, _ = timed(text_step, tsteps, max(1, args.warmup // 2))
        text = {"metric": "texts/sec embedding, ViT-B/32 text tower, batch 1024 x 77 tokens",
                "value": round(world * B_TEXT * tsteps / tdt, 1), "unit": "texts/s",
                "ms_per_step": round(tdt * 1e3 / tsteps, 3),
                "mfma_tflops": round(text_flops(B_TEXT, executed=True) * world * tsteps / tdt / 1e12 / world, 1)}
        text["frac_of_peak"] = round(text["mfma_tflops"] / PEAK_BF16_TFLOPS, 4)
        t_lanes = ctypes.c_int()
        _lib.check(_lib.lib().clipgpu_test_engine_lanes(te._h, ctypes.byref(t_lanes)))
        text["lanes"] = t_lanes.value
        tout_host = tout.cpu().numpy()
        if world == 1 and not args.no_e2e:
            ids_host = np.array(ids.cpu().numpy())  # a numpy-owned caller array, as a Rust caller's Vec
            text_e2e = {"text_ids_host": host_leg(te, "tokens", ids_host, max(5, args.steps // 2)),
                        "text_ids_host_registered": host_leg(te, "tokens", ids_host, max(5, args.steps // 2),
                                                             registered=True)}
        te.close()

    # End-to-end legs (host buffers in, host embeddings out, PCIe included; not `value`): the
    # reference's embed_images / embed_texts hand host arrays to the session (src/vision.rs:102-113,
    # src/text.rs:150-166); here through the C ABI's host entry points with pinned-staging overlap.
    e2e = None
    if world == 1 and not args.no_e2e:
        g = torch.Generator(device="cpu").manual_seed(1000 + rank)
        # numpy-owned caller arrays (copies out of torch's CPU allocator), as a Rust caller's buffers
        u8_host = np.array(torch.randint(0, 256, (B_VISION, 224, 224, 3), dtype=torch.uint8, generator=g).numpy())
        px_host = np.array(px.cpu().numpy())
        n_e2e = max(5, args.steps // 2)
        e2e = {"vision_u8_host": host_leg(ve, "u8", u8_host, n_e2e),
               "vision_u8_host_registered": host_leg(ve, "u8", u8_host, n_e2e, registered=True),
               "vision_f32_host": host_leg(ve, "f32", px_host, n_e2e),
               "vision_f32_host_registered": host_leg(ve, "f32", px_host, n_e2e, registered=True)}
        # four consecutive 256-image batches in one call: the engine alternates two staging sets, so
        # batch i + 1's host copy and H2D run under batch i's forward (engine.hip run_host_shard)
        u8_4x = np.concatenate([u8_host, np.roll(u8_host, 1, axis=0), np.roll(u8_host, 2, axis=0),
                                np.roll(u8_host, 3, axis=0)])
        e2e["vision_u8_host_4x256"] = host_leg(ve, "u8", u8_4x, max(2, n_e2e // 2))
        e2e["vision_u8_host_4x256_registered"] = host_leg(ve, "u8", u8_4x, max(2, n_e2e // 2), registered=True)
        u8_8x = np.concatenate([u8_4x, u8_4x[::-1]])
        e2e["vision_u8_host_8x256_registered"] = host_leg(ve, "u8", u8_8x, 3, registered=True)
        for k in ("vision_u8_host", "vision_u8_host_registered", "vision_u8_host_4x256",
                  "vision_u8_host_4x256_registered", "vision_u8_host_8x256_registered", "vision_f32_host",
                  "vision_f32_host_registered"):
            e2e[k]["vs_device_resident"] = round(e2e[k]["value"] / value, 3)
        del u8_4x, u8_8x
        # the drop-in entry point (decoded images of any size -> embeddings), GPU and host preprocessing
        g2 = np.random.default_rng(77)
        dec224 = [u8_host[i] for i in range(B_VISION)]
        dec640 = [g2.integers(0, 256, (480, 640, 3), dtype=np.uint8) for _ in range(B_VISION)]
        e2e["vision_rgb8_224_gpu"] = images_leg(ve, dec224, n_e2e)
        e2e["vision_rgb8_640x480_gpu"] = images_leg(ve, dec640, n_e2e)
        e2e["vision_rgb8_640x480_host_preprocess"] = images_leg(ve, dec640, max(2, n_e2e // 2), host_preprocess=True)
        del dec640
        if text is not None:
            e2e.update(text_e2e)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        vision_step()
        torch.cuda.synchronize()
        cpu = cpu_baseline(px.cpu().numpy(), ids.cpu().numpy(), out.cpu().numpy(), tout_host, fout_host)

    form = ("LayerNorm folded" if ln_fold else "") if dom == "c_fc" else f"{x_store} residual"
    traffic, traffic_src = (load_traffic(dom, sites[dom]["rows_per_launch"], ",".join(str(t) for t in tiles), form)
                            if not fp8 else (None, None))
    if rank == 0:
        line = {
            "metric": "images/sec embedding, ViT-B/32-224 vision tower, batch 256 per GPU",
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (seeded u8 images normalised with OpenAI mean/std; seeded weights)",
            "config": {"workload": "BASELINE.json configs[1]: ViT-B/32-224 VisionEmbedder, batch 256 "
                                   "synthetic 224x224 per GPU, device-resident input",
                       "global_batch": world * B_VISION, "seq_len": 50,
                       "parallelism": f"dp{world}, {dev_lanes.value} concurrent sub-batch lane(s)/GPU (committed MI355X tile table)" + (" + the engine's RCCL all-gather (ncclAllGather in the C ABI) of the [B,512] embeddings on every rank" if dp else "")},
            "roofline": {"bound": "mfma",
                         "kernel": f"{dom} GEMM ({sites[dom]['shape']}, {dom_epi}, tile {sites[dom]['tile']}): the "
                                   f"site with the most GEMM time per step",
                         "rows_per_launch": sites[dom]["rows_per_launch"],
                         "achieved": sites[dom]["tflops"], "peak": peak, "unit": "TFLOP/s",
                         "frac": sites[dom]["frac"], "traffic": traffic,
                         "traffic_source": traffic_src,
                         "launches_timed": site_prof[dom][1], "avg_launch_us": sites[dom]["avg_launch_us"],
                         "blocks": sites[dom]["blocks"],
                         "cu_frac": sites[dom]["concurrent"]["cu_frac"],
                         "cu_frac_note": "the same launches timed with both lanes running (CLIPGPU_PROFILE_CONCURRENT): "
                                         "FLOPs / (launch time x min(blocks, CUs) x the per-CU share of the peak); "
                                         "achieved / frac are the lanes-serialized launch (as rocprofv3 traces it)"},
            "gemm_cu_us_per_step": round(sum(v["concurrent"]["cu_us_per_step"] for v in sites.values()), 1),
            "gemm_sites": dict(sites, note="per-launch HIP-event times of each trunk GEMM site in a profiled pass "
                                           "(lanes serialized); us_per_step sums the site's launches; concurrent: the "
                                           "same with both lanes running, cu_us_per_step = its launches' time x "
                                           "min(blocks, CUs) / CUs (the CU time the site takes per step)"),
            "gemm_tiles": gemm_tiles,
            "gemm_tiles_env": ",".join(str(t) for t in tiles),
            "lanes_env": dev_lanes.value,
            "whole_forward_mfma_tflops_per_gpu": round(whole_tflops, 1),
            "whole_forward_frac_of_peak": round(whole_tflops / PEAK_BF16_TFLOPS, 4),
            "last_layer_pruned": PRUNE_LAST,
            "residual_stream": x_store,
            "ln_fold": ln_fold,
            "windows": windows,
            "sclk_mhz": windows["sclk_mhz_median"] if windows else None,
            **({"breakdown_serialized": breakdown} if breakdown is not None else {}),
            "text": text,
            "end_to_end": e2e,
            "fp8": fp8_info,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ve.close()
    if dp:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
