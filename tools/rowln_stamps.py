#!/usr/bin/env python3
"""Per-phase cycle breakdown of the fused residual GEMM + LayerNorm (gemm_rowln.hip) from the
diagnostic stamp build (make -C clip-embedder-rs_amd stamps).  Slots: 0 start, 1 prologue issued,
2+kt K-step kt done, 50 loop done, 51 residual stored, 52 mean, 53 variance, 54 end, 62/63 realtime.
SHAPES env "M,D,K;..." (default the ViT-B/32 trunk shapes), PF env (prefetch distance, default 8)."""
import ctypes
import os

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
lib = ctypes.CDLL(os.path.join(ROOT, "clip-embedder-rs_amd", "lib", "libclipgpu_stamps.so"))
lib.clipgpu_diag_rowln_stamps.argtypes = [ctypes.c_int] + [ctypes.c_int64] * 3 + [ctypes.c_int, ctypes.c_int,
                                                                                  ctypes.c_void_p, ctypes.c_int]
lib.clipgpu_last_error.restype = ctypes.c_char_p
NB = 2048
PF = int(os.environ.get("PF", "8"))
shapes = [tuple(map(int, t.split(","))) for t in os.environ.get(
    "SHAPES", "64,768,768;6400,768,768;12800,768,768;12800,768,3072").split(";")]

for M, D, K in shapes:
    for with_ln in (1, 0):
        buf = np.zeros((NB, 64), np.uint64)
        rc = lib.clipgpu_diag_rowln_stamps(0, M, D, K, PF, with_ln, buf.ctypes.data, NB)
        if rc:
            print("error", lib.clipgpu_last_error().decode())
            continue
        s = buf.astype(np.int64)
        s = s[s[:, 0] > 0]
        nk = K // 32
        last = 54 if with_ln else 51
        med = lambda a, b: float(np.median(s[:, b] - s[:, a]))  # noqa: E731
        steps = np.diff(s[:, 2:2 + min(nk, 40)], axis=1)
        real = float(np.median(s[:, 63] - s[:, 62])) * 10.0  # ns (100 MHz)
        cyc = float(np.median(s[:, last] - s[:, 0]))
        print(f"M{M} D{D} K{K} ln{with_ln} pf{PF}: blocks {len(s)}, block {cyc:.0f} cyc = {real / 1000:.2f} us "
              f"({cyc / max(real, 1):.2f} GHz) | prologue {med(0, 1):.0f} | step0 {med(1, 2):.0f} | "
              f"K-step p10/p50/p90 {np.percentile(steps, 10):.0f}/{np.median(steps):.0f}/{np.percentile(steps, 90):.0f}"
              f" | loop {med(1, 50):.0f} | resid {med(50, 51):.0f}"
              + (f" | mean {med(51, 52):.0f} | var {med(52, 53):.0f} | out {med(53, 54):.0f}" if with_ln else ""),
              flush=True)
