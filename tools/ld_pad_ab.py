#!/usr/bin/env python3
"""Row-pitch A/B of the trunk GEMMs: the same launch with A / W rows at pitch K and at K + pad.

The c_proj launch (A = the MLP hidden, rows of K = 3072 16-bit elements = 6 KiB) fetched 1.96x its
compulsory bytes at the two-lane table (profiles/pmc_c_fc.json), about 47 MB per launch beyond W's
per-XCD re-read.  If that excess is L2 set pressure from the 6 KiB row stride of the 224-row A panel
and the 192-row W panel, a padded pitch moves it; this script times both (alternating, median of
REPS) at the per-lane shapes of the ViT-B/32 bench.

usage: ld_pad_ab.py [REPS] [site ...]     sites: c_proj c_fc out_proj qkv (default all); LD_PADS=0,64 (pads)
       ld_pad_ab.py one SITE PAD ITERS    (one config, for rocprofv3 --pmc passes)
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

ROWS, D, MLP = 6400, 768, 3072
# site: (N, K, epi, act, tile) at the two-lane table (18, 26, 15, 26)
SITES = {"qkv": (3 * D, D, 0, 0, 18), "out_proj": (D, D, 1, 0, 26), "c_fc": (MLP, D, 0, 1, 15),
         "c_proj": (D, MLP, 1, 0, 26)}
PADS = tuple(int(x) for x in os.environ.get("LD_PADS", "0,64,32,8").split(","))


def run(site, pad, iters):
    N, K, epi, act, tile = SITES[site]
    us = ctypes.c_double()
    _lib.check(_lib.lib().clipgpu_test_gemm_bench_ld(0, epi, act, ROWS, N, K, K + pad, K + pad, tile, iters,
                                                     ctypes.byref(us)))
    return us.value


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        site, pad, iters = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
        print(f"{site} pad {pad}: {run(site, pad, iters):.2f} us", flush=True)
        return
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    sites = sys.argv[2:] or list(SITES)
    for site in sites:
        t = {p: [] for p in PADS}
        for _ in range(reps):
            for p in PADS:
                t[p].append(run(site, p, 30))
        rec = {"site": site, "rows": ROWS, "tile": SITES[site][4],
               "us_median": {str(p): round(statistics.median(v), 2) for p, v in t.items()},
               "us_all": {str(p): [round(x, 2) for x in v] for p, v in t.items()}}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
