#!/usr/bin/env python3
"""Where a poison-build GEMM output goes NaN (tile, shape): rows / columns hit.
usage: poison_diag.py tile[,tile] M,N,K,mode[;M,N,K,mode...]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
P = ctypes.CDLL(os.path.join(ROOT, "clip-embedder-rs_amd", "lib", "libclipgpu_poison.so"))
P.clipgpu_test_gemm.argtypes = [ctypes.c_int] * 3 + [ctypes.c_int64] * 3 + [ctypes.c_void_p] * 5
P.clipgpu_last_error.restype = ctypes.c_char_p
for t in sys.argv[1].split(","):
    os.environ["CLIPGPU_TEST_TILE"] = t
    for shp in sys.argv[2].split(";"):
        M, N, K, mode = (int(x) for x in shp.split(","))
        rng = np.random.default_rng(1)
        A = rng.standard_normal((M, K)).astype(np.float32)
        W = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
        bias = rng.standard_normal(N).astype(np.float32)
        resid = rng.standard_normal((M, N)).astype(np.float32)
        for rep in range(3):
            got = np.empty((M, N), np.float32)
            rc = P.clipgpu_test_gemm(0, mode, 0, M, N, K, A.ctypes.data, W.ctypes.data, bias.ctypes.data,
                                     resid.ctypes.data if mode == 1 else None, got.ctypes.data)
            assert rc == 0, P.clipgpu_last_error()
            bad = np.isnan(got)
            r, c = np.nonzero(bad)
            desc = "" if not len(r) else (f" rows {r.min()}-{r.max()} ({len(np.unique(r))}) cols {c.min()}-{c.max()} "
                                          f"({len(np.unique(c))}) colmod256 {sorted(set((np.unique(c) % 256) // 16))}")
            print(f"tile {t} {M}x{N}x{K} mode {mode} rep {rep}: nan {int(bad.sum())}{desc}", flush=True)
