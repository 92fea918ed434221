#!/usr/bin/env python3
"""Where a GEMM launch's time goes across its blocks (stamp build, lib/libclipgpu_stamps.so).

    python tools/gemm_stamp_dist.py M N K epi act tile [iters]

K <= 27 * 64 + 64 only (the K-step stamps of longer K reach slots 61-63 in builds before the
guard).  The stamp build records per block (wave 0): s_memrealtime at start / end (slots 62 / 63, one
100 MHz clock for the whole chip), s_memtime phase stamps (slots 0-5: per-XCD clock) and the
block's XCC_ID / HW_ID (slot 61).  Prints the launch span, the spread of block start times
(dispatch) and block durations, the durations split by how many blocks shared the block's CU
and by XCD, and the slowest blocks.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
lib = ctypes.CDLL(os.path.join(ROOT, "clip-embedder-rs_amd", "lib", "libclipgpu_stamps.so"))
lib.clipgpu_diag_gemm_stamps.argtypes = [ctypes.c_int] * 3 + [ctypes.c_int64] * 3 + [ctypes.c_int, ctypes.c_void_p,
                                                                                      ctypes.c_int, ctypes.c_int]
lib.clipgpu_last_error.restype = ctypes.c_char_p
NB = 2048

M, N, K, epi, act, tile = (int(x) for x in sys.argv[1:7])
iters = int(sys.argv[7]) if len(sys.argv) > 7 else 3


def pct(a, qs=(0, 10, 50, 90, 100)):
    return "/".join(f"{np.percentile(a, q):.1f}" for q in qs)


for it in range(iters):
    buf = np.zeros((NB, 64), np.uint64)
    rc = lib.clipgpu_diag_gemm_stamps(0, epi, act, M, N, K, tile, buf.ctypes.data, NB, 0)
    if rc:
        sys.exit("error " + lib.clipgpu_last_error().decode())
    used = buf[:, 63] > 0
    idx = np.nonzero(used)[0]
    s = buf[used].astype(np.int64)
    r0, r1 = s[:, 62], s[:, 63]
    t0 = r0.min()
    start = (r0 - t0) / 100.0  # µs
    end = (r1 - t0) / 100.0
    dur = end - start
    hw = s[:, 61] & 0xFFFFFFFF
    xcc = (s[:, 61] >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    uniq, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    share = cnt[inv]
    print(f"{M}x{N}x{K} epi{epi} tile {tile} run {it}: {len(s)} blocks on {len(uniq)} CUs, span {end.max():.1f} us")
    print(f"   start us (min/p10/p50/p90/max) {pct(start)} | duration {pct(dur)} | end {pct(end)}")
    for c in sorted(set(share.tolist())):
        sel = share == c
        print(f"   blocks on CUs holding {c} of this launch's blocks: {sel.sum():4d}, duration {pct(dur[sel])}, "
              f"start p50 {np.median(start[sel]):.1f}")
    per_x = " ".join(f"x{x}:{np.median(dur[xcc == x]):.1f}/{dur[xcc == x].max():.1f}({(xcc == x).sum()})"
                     for x in range(8) if (xcc == x).any())
    print(f"   per XCD duration p50/max(blocks): {per_x}")
    slow = np.argsort(-end)[:6]
    print("   latest-ending blocks: " + "; ".join(
        f"b{idx[i]} x{xcc[i]} se{se[i]} cu{cu[i]} share{share[i]} start {start[i]:.1f} dur {dur[i]:.1f}" for i in slow))
    sys.stdout.flush()
