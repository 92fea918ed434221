#!/usr/bin/env python3
"""Median per-dispatch counter values from rocprofv3 --pmc counter_collection CSVs.
usage: pmc_summary.py DIR_PREFIX [KERNEL_SUBSTRING]  (every DIR_PREFIX* directory)"""
import collections
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "gemm"
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(d + "*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if pat in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    print(f"{k:32s} n={len(vals[k]):4d} median={statistics.median(vals[k]):.4g}")
