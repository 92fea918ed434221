#!/usr/bin/env python3
"""Timeline of the registered-u8 host path (run under rocprofv3 --kernel-trace --memory-copy-trace):
ViT-B/32 bf16, max_batch 256, u8 [256,224,224,3] registered input/output, CALLS calls 20 ms apart
(so each call is its own cluster in the trace).  `host_trace.py analyze DIR` prints per call: the H2D
copies (start / end relative to the call's first operation, GB/s), each lane's first kernel start and
last kernel end, the D2H copies and the span."""
import glob
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def run(calls):
    import numpy as np
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
    from open_clip_inference.engine import Engine, host_register  # noqa: E402
    from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, VIT_B_32_CFG  # noqa: E402
    from tests.helpers import make_model_dir  # noqa: E402
    B = 256
    e = Engine(make_model_dir(VIT_B_32_CFG, 1234), 0, [0], "bf16", B)
    x = np.ascontiguousarray(np.random.default_rng(5).integers(0, 256, (B, 224, 224, 3), dtype=np.uint8))
    out = np.empty((B, 512), np.float32)
    host_register(x)
    host_register(out)
    for _ in range(3):
        e.embed_u8(x, OPENAI_MEAN, OPENAI_STD, out=out)
    for _ in range(calls):
        time.sleep(0.02)
        t0 = time.perf_counter()
        e.embed_u8(x, OPENAI_MEAN, OPENAI_STD, out=out)
        print(f"call {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)


def analyze(d):
    import csv
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r.get("Stream_Id", r.get("Queue_Id", "?")),
                         r["Kernel_Name"][:40], 0))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", "?"),
                         r.get("Direction", ""), int(r.get("Size", r.get("Bytes", 0)) or 0)))
    rows.sort()
    calls, cur, last = [], [], None
    for r in rows:
        if last is not None and r[0] - last > 5_000_000:
            calls.append(cur)
            cur = []
        cur.append(r)
        last = max(last or 0, r[1])
    calls.append(cur)
    for c in calls[-6:]:
        t0 = c[0][0]
        span = (max(r[1] for r in c) - t0) / 1e3
        print(f"--- call: {len(c)} ops, span {span:.1f} us")
        for r in c:
            if r[2] == "C":
                gbps = r[5] / max(1, r[1] - r[0])
                print(f"  copy {r[3]:>14} {r[5] / 1e6:7.2f} MB  {(r[0] - t0) / 1e3:8.1f} .. {(r[1] - t0) / 1e3:8.1f} us  {gbps:.1f} GB/s")
        streams = {}
        for r in c:
            if r[2] == "K":
                s = streams.setdefault(r[3], [r[0], r[1], 0])
                s[0], s[1], s[2] = min(s[0], r[0]), max(s[1], r[1]), s[2] + 1
        for k, (a, b, n) in sorted(streams.items(), key=lambda kv: kv[1][0]):
            print(f"  stream {k}: {n} kernels {(a - t0) / 1e3:8.1f} .. {(b - t0) / 1e3:8.1f} us")


if __name__ == "__main__":
    if sys.argv[1] == "analyze":
        analyze(sys.argv[2])
    else:
        run(int(sys.argv[1]))
