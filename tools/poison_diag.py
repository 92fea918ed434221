#!/usr/bin/env python3
"""Where a poison-build GEMM output goes NaN or wrong (tile, shape): rows / columns hit.

usage: poison_diag.py tile[,tile] M,N,K,mode[;M,N,K,mode...] [reps]
  CLIPGPU_POISON_LIB  the race-check library (default lib/libclipgpu_poison.so)
  CLIPGPU_REF_LIB     the same sources without the poison (default lib/libclipgpu.so): each run's
                      output is also compared bit for bit with it, so a wrong-but-finite result
                      (a stale tile) is reported too.
mode: 0 = 16-bit store, 1 = f32 residual, 2 = f32 store (clipgpu_test_gemm).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "clip-embedder-rs_amd", "lib")


def load(path):
    L = ctypes.CDLL(path)
    L.clipgpu_test_gemm.argtypes = [ctypes.c_int] * 3 + [ctypes.c_int64] * 3 + [ctypes.c_void_p] * 5
    L.clipgpu_last_error.restype = ctypes.c_char_p
    return L


P = load(os.environ.get("CLIPGPU_POISON_LIB", os.path.join(LIBDIR, "libclipgpu_poison.so")))
R = load(os.environ.get("CLIPGPU_REF_LIB", os.path.join(LIBDIR, "libclipgpu.so")))
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3


def run(L, M, N, K, mode, A, W, bias, resid):
    got = np.full((M, N), -7.0, np.float32)
    rc = L.clipgpu_test_gemm(0, mode, 0, M, N, K, A.ctypes.data, W.ctypes.data, bias.ctypes.data,
                             resid.ctypes.data if mode == 1 else None, got.ctypes.data)
    assert rc == 0, L.clipgpu_last_error()
    return got


def desc(mask):
    r, c = np.nonzero(mask)
    if not len(r):
        return "none"
    return (f"{int(mask.sum())} elems rows {r.min()}-{r.max()} ({len(np.unique(r))}) rows mod tile "
            f"{sorted(set(np.unique(r) % 224))[:12]} cols {c.min()}-{c.max()} ({len(np.unique(c))}) "
            f"col blocks/16 mod 256 {sorted(set((np.unique(c) % 256) // 16))}")


for t in sys.argv[1].split(","):
    os.environ["CLIPGPU_TEST_TILE"] = t
    for shp in sys.argv[2].split(";"):
        M, N, K, mode = (int(x) for x in shp.split(","))
        rng = np.random.default_rng(1)
        A = rng.standard_normal((M, K)).astype(np.float32)
        W = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
        bias = rng.standard_normal(N).astype(np.float32)
        resid = rng.standard_normal((M, N)).astype(np.float32)
        ref = run(R, M, N, K, mode, A, W, bias, resid)
        for rep in range(reps):
            got = run(P, M, N, K, mode, A, W, bias, resid)
            nan = np.isnan(got)
            diff = (got != ref) & ~nan
            print(f"tile {t} {M}x{N}x{K} mode {mode} rep {rep}: nan: {desc(nan)} | wrong finite: {desc(diff)}",
                  flush=True)
