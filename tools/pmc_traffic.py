#!/usr/bin/env python3
"""HBM traffic per launch of a vision trunk GEMM from two rocprofv3 --pmc passes.

Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON ROWS_PER_LAUNCH SOURCE_LABEL TILES [SITE]

SITE: c_fc (default), c_proj or out_proj.  TILES: the engine's gemm_tiles_env of the profiled run
("q,o,f,p"); bench.py only takes a record whose tiles equal its own run's.

FETCH_DIR / WRITE_DIR hold `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`
counter_collection CSVs of the same `bench.py --no-text` command (separate passes: the
two counters cannot share one on gfx950).  Per MI355X_MICROARCH.md §HBM: both counters
are in KB; FETCH_SIZE reports half the bytes of wide coalesced streaming reads on gfx950,
so it is doubled; WRITE_SIZE is exact for 16-byte-per-lane stores.

Kernels (vision leg, bf16):
- c_fc: gemm_{bt,pipe}_kernel<T, ..., EPI_STORE16 = 0, ACT_QUICK_GELU = 1> (the only launch with an
  activation);
- out_proj / c_proj: the residual launches gemm_{bt,pipe}_kernel<T, ..., EPI_RESID = 1, ACT_NONE = 0>.
  Both sites run that kernel; c_proj reads its K = 4 D operand (4x out_proj's A), so in the
  FETCH_SIZE pass the residual dispatches split into two clusters and the upper one is c_proj.  The
  WRITE_SIZE pass (both write the same f32 x rows) is classified by dispatch order: both passes
  run the same command, so the i-th residual dispatch is the same launch in both.
Compulsory bytes per launch: A + W (16-bit) + bias + output (c_fc: 16-bit hidden) or the f32
residual read and write (out_proj / c_proj).
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

KERNELS = {
    # c_fc: EPI_STORE16 (bf16 operands) or, LayerNorm-folded, EPI_LNF_BF = 8 (f16 operands); QuickGELU
    "c_fc": re.compile(r"gemm_(bt|pipe)_kernelIDF16(?:b|_)Li\d+ELi\d+ELi\d+ELi\d+ELi(?:0|8)ELi1E(?:Li\d+E)*EEv"),
    # out_proj / c_proj: EPI_RESID = 1 (f32 stream) or EPI_RESID16 = 5 (f16 stream)
    "resid": re.compile(r"gemm_(bt|pipe)_kernelIDF16bLi\d+ELi\d+ELi\d+ELi\d+ELi(?:1|5)ELi0E(?:Li\d+E)*EEv"),
}
D, MLP = 768, 3072  # ViT-B/32 vision
SHAPES = {"c_fc": (MLP, D), "c_proj": (D, MLP), "out_proj": (D, D)}  # (N, K)


NAMES = set()  # the matched kernel names (the epilogue forms the compulsory bytes follow)


def dispatches(d, counter, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter and pattern.search(row["Kernel_Name"]):
                    out.append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
                    NAMES.add(pattern.search(row["Kernel_Name"]).group(0))
    out.sort()
    return [v for _, v in out]


def site_values(site, fetch_dir, write_dir):
    if site == "c_fc":
        f = dispatches(fetch_dir, "FETCH_SIZE", KERNELS["c_fc"])
        w = dispatches(write_dir, "WRITE_SIZE", KERNELS["c_fc"])
        return f, w
    f = dispatches(fetch_dir, "FETCH_SIZE", KERNELS["resid"])
    w = dispatches(write_dir, "WRITE_SIZE", KERNELS["resid"])
    if not f or len(f) != len(w):
        raise SystemExit(f"residual dispatches differ between the passes ({len(f)} vs {len(w)})")
    cut = (min(f) + max(f)) / 2
    upper = site == "c_proj"
    idx = [i for i, v in enumerate(f) if (v > cut) == upper]
    return [f[i] for i in idx], [w[i] for i in idx]


def main():
    fetch_dir, write_dir, out, rows, label, tiles = sys.argv[1:7]
    site = sys.argv[7] if len(sys.argv) > 7 else "c_fc"
    M = int(rows)
    fv, wv = site_values(site, fetch_dir, write_dir)
    if not fv or not wv:
        raise SystemExit(f"no {site} dispatches under {fetch_dir} / {write_dir}")
    f_kb, w_kb = statistics.median(fv), statistics.median(wv)
    read_b, write_b = 2.0 * f_kb * 1024.0, w_kb * 1024.0
    N, K = SHAPES[site]
    if site == "c_fc":
        lnf = any("ELi8ELi1E" in n for n in NAMES)
        if lnf:  # + the column sums (f32) and the rows' (mean, rstd)
            compulsory, what = 2 * (M * K + N * K + M * N) + 8 * N + 8 * M, "LayerNorm folded, +QuickGELU"
        else:
            compulsory, what = 2 * (M * K + N * K + M * N) + 4 * N, "+QuickGELU"
    else:
        xb = 2 if any("ELi5ELi0E" in n for n in NAMES) else 4
        compulsory = 2 * (M * K + N * K) + 4 * N + 2 * xb * M * N
        what = f"+bias, {'f16' if xb == 2 else 'f32'} residual read and write"
    res = {
        "kernel": f"{site} GEMM ({M}x{N}x{K}, bf16, {what})", "site": site, "rows_per_launch": M,
        "fetch_size_kb_median": f_kb, "write_size_kb_median": w_kb,
        "fetch_dispatches": len(fv), "write_dispatches": len(wv),
        "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b, "source": label,
        "compulsory_bytes_per_launch": compulsory,
        "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), KB x 1024; WRITE_SIZE as reported",
        "tiles": tiles,
    }
    # one record per (site, rows per launch), merged into OUT_JSON's "by_rows" (c_fc, the historical
    # keys) / "by_site_rows" ("site:rows"); the latest also at the top level
    prev = {}
    if os.path.exists(out):
        with open(out) as fh:
            prev = json.load(fh)
    by_rows = prev.get("by_rows", {})
    by_site = prev.get("by_site_rows", {})
    if site == "c_fc":
        by_rows[str(M)] = res
    by_site[f"{site}:{M}"] = res
    res = dict(res, by_rows=by_rows, by_site_rows=by_site)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("by_rows", "by_site_rows")}))


if __name__ == "__main__":
    main()
