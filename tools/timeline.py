#!/usr/bin/env python3
"""Per-launch timeline of the concurrent-lane forward (diagnostic).

Runs the bench's vision (B = 256) or text (B = 1024 x 77) engine with every profile category on and
CLIPGPU_PROFILE_CONCURRENT (the lanes stay concurrent; graphs off), then reads each launch's start /
end / category / lane (clipgpu_test_profile_timeline) and reports, per kernel class:
  - mean duration, and mean duration split by what the other lane was running most of the time;
  - each lane's idle time between its kernels (dispatch gaps + waits);
  - the busy-time union of both lanes vs the step time.
Writes gpurun_out/timeline_<tower>.json (summary) and gpurun_out/timeline_<tower>_raw.json (launches).
Usage: python tools/timeline.py [vision|text] [steps] [lanes]
"""
import collections
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))

import bench  # noqa: E402
from open_clip_inference import _lib  # noqa: E402
from open_clip_inference.engine import PROFILE_CATEGORIES, Engine, profile_enable  # noqa: E402


def main():
    tower = sys.argv[1] if len(sys.argv) > 1 else "vision"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    lanes = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    mdir = bench.make_model_dir()
    px, ids = bench.synth_inputs(0, dev)
    stream = torch.cuda.current_stream(dev)
    if tower == "vision":
        eng = Engine(mdir, _lib.TOWER_VISION, [0], "bf16", bench.B_VISION, lanes=lanes)
        out = torch.empty((bench.B_VISION, 512), device=dev)

        def step():
            eng.embed_pixels_device(px.data_ptr(), bench.B_VISION, out.data_ptr(), stream.cuda_stream)
    else:
        eng = Engine(mdir, _lib.TOWER_TEXT, [0], "bf16", bench.B_TEXT, lanes=lanes)
        out = torch.empty((bench.B_TEXT, 512), device=dev)

        def step():
            eng.embed_tokens_device(ids.data_ptr(), bench.B_TEXT, out.data_ptr(), stream.cuda_stream)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    profile_enable(eng, PROFILE_CATEGORIES, concurrent=True)
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    n_max = 20000
    t0 = (ctypes.c_double * n_max)()
    t1 = (ctypes.c_double * n_max)()
    cat = (ctypes.c_int * n_max)()
    lane = (ctypes.c_int * n_max)()
    n = ctypes.c_int64()
    _lib.check(_lib.lib().clipgpu_test_profile_timeline(eng.handle, n_max, t0, t1, cat, lane, ctypes.byref(n)))
    profile_enable(eng, [])
    m = min(n.value, n_max)
    recs = [{"t0": t0[i], "t1": t1[i], "cat": PROFILE_CATEGORIES[cat[i]], "lane": lane[i]} for i in range(m)]
    os.makedirs("gpurun_out", exist_ok=True)
    tag = f"{tower}" + (f"_l{lanes}" if lanes else "")
    with open(f"gpurun_out/timeline_{tag}_raw.json", "w") as f:
        json.dump(recs, f)
    print(json.dumps(summarize(recs, steps)), flush=True)
    with open(f"gpurun_out/timeline_{tag}.json", "w") as f:
        json.dump(summarize(recs, steps), f, indent=1)
    eng.close()


def summarize(recs, steps):
    span = max(r["t1"] for r in recs) - min(r["t0"] for r in recs)
    by_lane = collections.defaultdict(list)
    for r in recs:
        by_lane[r["lane"]].append(r)
    lanes = {}
    for ln, rs in by_lane.items():
        rs.sort(key=lambda r: r["t0"])
        busy = sum(r["t1"] - r["t0"] for r in rs)
        gaps = [max(0.0, b["t0"] - a["t1"]) for a, b in zip(rs, rs[1:])]
        lanes[str(ln)] = {"launches": len(rs), "busy_ms": round(busy, 3), "gap_ms": round(sum(gaps), 3),
                          "gap_median_us": round(1e3 * float(np.median(gaps)), 2) if gaps else None}
    # union of busy intervals over both lanes
    iv = sorted((r["t0"], r["t1"]) for r in recs)
    union, cur0, cur1 = 0.0, None, None
    for a, b in iv:
        if cur1 is None or a > cur1:
            if cur1 is not None:
                union += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    union += cur1 - cur0
    # per class: durations, split by the other lane's dominant class during the launch
    other = {}
    for ln, rs in by_lane.items():
        other[ln] = [r for l2, rr in by_lane.items() if l2 != ln for r in rr]
    cls = collections.defaultdict(lambda: {"n": 0, "ms": 0.0, "beside": collections.defaultdict(lambda: [0, 0.0])})
    for ln, rs in by_lane.items():
        for r in rs:
            d = r["t1"] - r["t0"]
            c = cls[r["cat"]]
            c["n"] += 1
            c["ms"] += d
            ov = collections.defaultdict(float)
            for o in other[ln]:
                x = min(r["t1"], o["t1"]) - max(r["t0"], o["t0"])
                if x > 0:
                    ov[o["cat"]] += x
            dom = max(ov, key=ov.get) if ov and max(ov.values()) > 0.5 * d else "idle/gap"
            c["beside"][dom][0] += 1
            c["beside"][dom][1] += d
    out = {"steps": steps, "span_ms": round(span, 3), "ms_per_step": round(span / steps, 3),
           "busy_union_ms_per_step": round(union / steps, 3), "lanes": lanes, "classes": {}}
    for k, c in sorted(cls.items(), key=lambda kv: -kv[1]["ms"]):
        out["classes"][k] = {"launches_per_step": c["n"] / steps, "ms_per_step": round(c["ms"] / steps, 3),
                             "mean_us": round(1e3 * c["ms"] / c["n"], 2),
                             "beside": {b: {"n": v[0], "mean_us": round(1e3 * v[1] / v[0], 2)}
                                        for b, v in sorted(c["beside"].items(), key=lambda kv: -kv[1][0])}}
    return out


if __name__ == "__main__":
    main()
