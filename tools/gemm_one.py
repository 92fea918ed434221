#!/usr/bin/env python3
"""Run one GEMM config repeatedly (for rocprofv3 PMC passes) or a small sweep.
usage: gemm_one.py M N K epi act tile iters"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

M, N, K, epi, act, tile, iters = (int(x) for x in sys.argv[1:8])
us = ctypes.c_double()
_lib.check(_lib.lib().clipgpu_test_gemm_bench(0, epi, act, M, N, K, tile, iters, ctypes.byref(us)))
print(f"{M}x{N}x{K} epi{epi} act{act} tile{tile}: {us.value:.2f} us  {2.0*M*N*K/us.value/1e6:.1f} TF/s", flush=True)
