#!/usr/bin/env python3
"""Per-phase cycle breakdown of the GEMM tile loop from the diagnostic stamp build.

    make -C clip-embedder-rs_amd stamps && python tools/gemm_stamps.py

Loads lib/libclipgpu_stamps.so (s_memtime stamps of wave 0 of every block, see gemm.hip
GEMM_STAMP slots: 0 start, 1 prologue done, 2+4i tile i start, 3+4i main loop done,
4+4i last K-step done, 5+4i epilogue done, 34+kt K-step kt of tile 0 done, 62/63 realtime).
Stamps cost a few % of wave time; compare phases, not absolute TF/s.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
lib = ctypes.CDLL(os.path.join(ROOT, "clip-embedder-rs_amd", "lib", "libclipgpu_stamps.so"))
lib.clipgpu_diag_gemm_stamps.argtypes = [ctypes.c_int] * 3 + [ctypes.c_int64] * 3 + [ctypes.c_int, ctypes.c_void_p,
                                                                                      ctypes.c_int, ctypes.c_int]
DIAG = int(os.environ.get("STAMP_DIAG", "0"))
lib.clipgpu_last_error.restype = ctypes.c_char_p
NB = 2048

# (name, epi (0 store16, 1 residual f32, 3 residual f16), act, M, N, K, tile): the committed table's
# tiles (engine.hip table_tiles) at the bench's two-lane rows (6400 per lane) and at one lane's 12800
CASES = [
    ("t26_c_proj 224x192w8", 3, 0, 6400, 768, 3072, 26),
    ("t26_out 224x192w8", 3, 0, 6400, 768, 768, 26),
    ("t15_c_fc 160x128rs", 0, 1, 6400, 3072, 768, 15),
    ("t18_qkv 256x256half", 0, 0, 6400, 2304, 768, 18),
    ("t15_c_proj 160x128rs", 3, 0, 6400, 768, 3072, 15),
    ("t26_c_proj_12800 224x192w8", 3, 0, 12800, 768, 3072, 26),
    ("t18_c_fc_12800 256x256half", 0, 1, 12800, 3072, 768, 18),
    ("square8k 256x256", 0, 0, 8192, 8192, 8192, 3),
]
if len(sys.argv) > 1:
    CASES = [c for c in CASES if any(a in c[0] for a in sys.argv[1:])]

for name, epi, act, M, N, K, tile in CASES:
    buf = np.zeros((NB, 64), np.uint64)
    rc = lib.clipgpu_diag_gemm_stamps(0, epi, act, M, N, K, tile, buf.ctypes.data, NB, DIAG)
    if rc:
        print(name, "error", lib.clipgpu_last_error().decode())
        continue
    s = buf.astype(np.int64)
    used = s[:, 1] > 0
    s = s[used]
    nb = len(s)
    nk = K // 64
    t0 = s[:, 0].min()
    # tiles per block
    ntile = np.array([sum(1 for i in range(8) if row[5 + 4 * i] > 0) for row in s])
    prol = np.median(s[:, 1] - s[:, 0])
    mains, lasts, epis, gaps = [], [], [], []
    for row, nt in zip(s, ntile):
        for i in range(nt):
            b = 2 + 4 * i
            mains.append(row[b + 1] - row[b])
            lasts.append(row[b + 2] - row[b + 1])
            epis.append(row[b + 3] - row[b + 2])
            if i + 1 < nt:
                gaps.append(row[b + 4] - row[b + 3])
    ks = np.diff(s[:, 34:min(34 + nk - 1, 61)], axis=1) if nk > 2 else np.zeros((nb, 0))  # slots 34..60
    end = np.array([row[5 + 4 * (nt - 1)] for row, nt in zip(s, ntile)])
    real = (s[:, 63] - s[:, 62]).astype(np.float64)
    cyc = (end - s[:, 0]).astype(np.float64)
    clk = np.median(cyc / np.maximum(real, 1) * 100.0)  # MHz (memtime ticks per realtime 10 ns)
    span = (end.max() - t0)
    flops = 2.0 * M * N * K
    print(f"{name:18s} M{M} N{N} K{K} diag{DIAG}: blocks {nb}, tiles/block "
          f"{np.bincount(ntile).nonzero()[0].tolist()}, block cycles p50/max {np.median(cyc):.0f}/{cyc.max():.0f} "
          f"(s_memtime is per XCD: only intra-block differences are meaningful)")
    print(f"    prologue {prol:7.0f} cyc | main loop ({nk - 1} K-steps) {np.median(mains):7.0f} "
          f"({np.median(mains) / max(nk - 1, 1):.0f}/step, K-step p10/p50/p90 "
          f"{np.percentile(ks, 10) if ks.size else 0:.0f}/{np.median(ks) if ks.size else 0:.0f}/"
          f"{np.percentile(ks, 90) if ks.size else 0:.0f}) | last step {np.median(lasts):6.0f} | "
          f"epilogue+sync {np.median(epis):6.0f}", flush=True)
