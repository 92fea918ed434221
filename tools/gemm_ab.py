#!/usr/bin/env python3
"""Interleaved A/B of GEMM tiles at one shape, in one process (cdna_hip_programming.md §5.4
rule 24): ROUNDS rounds, every tile once per round, median and min µs per tile.
usage: gemm_ab.py M N K epi act tile[,tile...] [rounds] [iters]
epi: 0 store16 (+act), 1 residual f32, 2 store32, 3 residual f16; tiles: kernels.hpp GemmTile ids."""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

M, N, K, epi, act = (int(x) for x in sys.argv[1:6])
tiles = [int(t) for t in sys.argv[6].split(",")]
rounds = int(sys.argv[7]) if len(sys.argv) > 7 else 5
iters = int(sys.argv[8]) if len(sys.argv) > 8 else 20
L = _lib.lib()
got = {t: [] for t in tiles}
for _ in range(rounds):
    for t in tiles:
        us = ctypes.c_double()
        _lib.check(L.clipgpu_test_gemm_bench(0, epi, act, M, N, K, t, iters, ctypes.byref(us)))
        got[t].append(us.value)
for t in tiles:
    med, mn = statistics.median(got[t]), min(got[t])
    print(f"{M}x{N}x{K} epi{epi} act{act} tile {t:3d}: median {med:8.2f} us  min {mn:8.2f} us  "
          f"{2.0 * M * N * K / med / 1e6:7.1f} TF/s (median)", flush=True)
