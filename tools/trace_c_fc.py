#!/usr/bin/env python3
"""Per-phase c_fc GEMM durations from a rocprofv3 --kernel-trace of `bench.py` (vision leg).

Usage: python tools/trace_c_fc.py KERNEL_TRACE_CSV STEPS WARMUP
Phases in launch order: autotune (3 tiles x 5 launches), warmup, timed loop (lanes
concurrent), profiling warmup + profiling pass (lanes serialized) — 12 layers x 2 lanes
c_fc launches per step.  The profiling-pass mean is what bench.py's HIP events report.
"""
import csv
import re
import statistics
import sys

path, steps, warmup = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
fc = [r for r in rows if re.search(r"gemm_bt_kernel.*Li0ELi0ELi1EEEv", r["Kernel_Name"])]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in fc]
per = 24
segs = [("autotune", 15), ("warmup", warmup * per), ("timed (lanes concurrent)", steps * per),
        ("profiling warmup", per), ("profiling pass (lanes serialized)", max(3, steps // 2) * per)]
i = 0
for name, n in segs:
    x = d[i:i + n]
    i += n
    print(f"{name:36s} launches {len(x):4d}  mean {statistics.mean(x):8.2f} us  median {statistics.median(x):8.2f} us")
