#!/usr/bin/env python3
"""Per-site launch durations of the residual GEMM kernel in a rocprofv3 kernel trace.

usage: site_split.py KERNEL_TRACE_CSV [SYMBOL_SUBSTRING] [OUT]

out_proj and c_proj run the same gemm_pipe_kernel instantiation (tile 26, EPI_RESID), so the
`--stats` summary averages both sites and both timing regimes of bench.py: the timed windows (two
lanes overlapping) and the profiled pass that times each launch alone (bench.py `gemm_sites` /
`roofline.avg_launch_us`).  This splits the launches by duration (2-means: c_proj has 4x out_proj's
K) and by isolation (no other kernel overlaps the launch = the profiled pass), so the bench's
`roofline.avg_launch_us` can be checked against the trace."""
import bisect
import csv
import json
import statistics
import sys


def main():
    path = sys.argv[1]
    sym = sys.argv[2] if len(sys.argv) > 2 else "Li224ELi192ELi2ELi4ELi1ELi0ELi3"
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))]
    rows.sort()
    starts = [r[0] for r in rows]
    ends_prefix_max = []
    m = 0
    for r in rows:
        m = max(m, r[1])
        ends_prefix_max.append(m)
    sel = [i for i, r in enumerate(rows) if sym in r[2]]
    dur = [(rows[i][1] - rows[i][0]) / 1e3 for i in sel]
    lo, hi = min(dur), max(dur)
    for _ in range(20):  # 2-means on the durations
        cut = (lo + hi) / 2
        a = [d for d in dur if d <= cut] or [cut]
        b = [d for d in dur if d > cut] or [cut]
        lo, hi = statistics.mean(a), statistics.mean(b)
    cut = (lo + hi) / 2

    def isolated(i):
        s, e = rows[i][0], rows[i][1]
        # an earlier-starting kernel still running, or a later one starting before this one ends
        if i > 0 and ends_prefix_max[i - 1] > s:
            return False
        j = bisect.bisect_left(starts, e)
        return not any(k != i for k in range(i + 1, j))

    out = {"trace": path, "symbol": sym, "duration_cut_us": round(cut, 2)}
    for site, pick in (("out_proj", lambda d: d <= cut), ("c_proj", lambda d: d > cut)):
        idx = [i for i, d in zip(sel, dur) if pick(d)]
        alone = [(rows[i][1] - rows[i][0]) / 1e3 for i in idx if isolated(i)]
        conc = [(rows[i][1] - rows[i][0]) / 1e3 for i in idx if not isolated(i)]
        out[site] = {"launches": len(idx),
                     "alone": {"n": len(alone), "mean_us": round(statistics.mean(alone), 2) if alone else None},
                     "beside_other_kernels": {"n": len(conc),
                                              "mean_us": round(statistics.mean(conc), 2) if conc else None}}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")


if __name__ == "__main__":
    main()
