#!/usr/bin/env python3
"""Per-kernel statistics of bench.py's timed steps only, from a rocprofv3 --kernel-trace CSV.

    python tools/trace_timed.py RUN_kernel_trace.csv STEPS [OUT.txt] [LANES]

For a vision-only bench (`--no-text --no-fp8 --no-e2e --no-cpu-baseline`): after the engine's
creation-time tuning, the trace ends with W warmup steps, the STEPS timed steps, then the c_fc
profiling pass (1 warmup + P = max(3, STEPS // 2) steps, lanes serialized), then the same P + 1
steps with the lanes concurrent (the concurrent site profile; skipped when finding the period).  Every step issues the
same kernel sequence, so the launches per step n is the period of the trace's tail; the timed
block is the STEPS * n launches before the last (P + 1) * n.  With LANES concurrent lanes the
profiling pass runs them one after the other, so the tail's period is one lane's forward and a
step is LANES * n launches; kernel durations in the timed block then overlap (the summed kernel
time per step exceeds the wall time per step).  Prints per-kernel calls per step,
mean / median duration and the share of the summed kernel time, plus the timed block's wall time
per step (first start to last end), so rocprof's numbers exclude the creation-time tuning launches
that rocprofv3 --stats mixes in.
"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def short(name):
    if not name.startswith("_Z"):  # demangled: "void ns::(anonymous namespace)::kernel<...>(...)"
        m = re.search(r"::(\w+)(<[^(]*>)?\(", name)
        return (m.group(1) + (m.group(2) or "")).replace(" ", "")[:60] if m else name[:60]
    m = re.search(r"N_1\d*(\w+?)I", name)
    base = m.group(1) if m else name[:40]
    args = re.findall(r"Li(\d+)E", name)
    return f"{base}<{','.join(args)}>" if args else base


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    lanes = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    names = [r[2] for r in rows]
    prof_steps = max(3, steps // 2) + 1
    n = None
    for cand in range(8, 2000):
        # the serialized pass ends where the concurrent pass (prof_steps steps of cand * lanes
        # launches, its lanes interleaved in start order) begins
        e = len(names) - prof_steps * cand * lanes
        if e >= 3 * cand and names[e - cand:e] == names[e - 2 * cand:e - cand] == names[e - 3 * cand:e - 2 * cand]:
            n = cand
            break
    if n is None:
        raise SystemExit("no periodic tail: not a vision-only bench trace?")
    n *= lanes  # launches per step
    end = len(rows) - 2 * prof_steps * n
    timed = rows[end - steps * n:end]
    out = [f"# {path}: {len(rows)} launches, {n} per step ({lanes} lane(s)); timed block = {steps} steps "
           f"({len(timed)} launches) before the {prof_steps}-step profiling pass",
           f"# timed block wall time per step (first start -> last end): "
           f"{(timed[-1][1] - timed[0][0]) / steps / 1e3:.1f} us; summed kernel time per step "
           f"{sum(e - s for s, e, _ in timed) / steps / 1e3:.1f} us"]
    per = defaultdict(list)
    for s, e, nm in timed:
        per[nm].append((e - s) / 1e3)
    tot = sum(sum(v) for v in per.values())
    out.append(f"{'kernel':60s} {'calls/step':>10s} {'mean_us':>9s} {'median_us':>9s} {'us/step':>9s} {'share':>6s}")
    for nm, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        out.append(f"{short(nm):60s} {len(v) / steps:10.1f} {statistics.mean(v):9.2f} {statistics.median(v):9.2f} "
                   f"{sum(v) / steps:9.1f} {sum(v) / tot:6.3f}")
    text = "\n".join(out)
    print(text)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
