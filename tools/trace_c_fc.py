#!/usr/bin/env python3
"""Per-phase c_fc GEMM durations from a rocprofv3 --kernel-trace of `bench.py` (vision leg).

Usage: python tools/trace_c_fc.py KERNEL_TRACE_CSV STEPS WARMUP

The vision c_fc launches are the QuickGELU GEMM dispatches (gemm_{bt,pipe}_kernel<..., EPI 0,
ACT 1>) up to the vision leg's last head kernel (the text engine's autotune follows it).  In launch order: autotune (candidate tiles x 5
launches), warmup, timed loop (lanes concurrent), profiling warmup + profiling pass (lanes
serialized) -- 12 layers x 2 lanes c_fc launches per step.  With the last layer pruned to the
pooled rows (clipgpu_options.prune_last, default on) its c_fc runs at M = 128 rows on the skinny
kernel, which the pattern does not match: 11 x 2 launches per step.  The profiling-pass mean is what
bench.py's HIP events report as roofline.avg_launch_us; this prints it from the trace so the
two can be compared.
"""
import csv
import re
import statistics
import sys

path, steps, warmup = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
text0 = next((i for i, r in enumerate(rows) if "text_embed_ln" in r["Kernel_Name"]), len(rows))
# the vision leg ends with its last head kernel (l2norm) before the text engine's autotune
vis_end = max(i for i, r in enumerate(rows[:text0]) if "l2norm_kernel" in r["Kernel_Name"]) + 1
fc_re = re.compile(r"gemm_(bt|pipe)_kernelIDF16bLi\d+ELi\d+ELi\d+ELi\d+ELi0ELi1E(?:Li\dE)?EEv")
fc = [r for r in rows[:vis_end] if fc_re.search(r["Kernel_Name"])]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in fc]
per = 22  # the last layer is pruned (the engine default)
n_prof = max(3, steps // 2) * per
segs = [("timed (lanes concurrent)", d[-(n_prof + per + steps * per):-(n_prof + per)]),
        ("profiling pass (lanes serialized)", d[-n_prof:])]
for name, x in segs:
    print(f"{name:36s} launches {len(x):4d}  mean {statistics.mean(x):8.2f} us  median {statistics.median(x):8.2f} us")
