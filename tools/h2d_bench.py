#!/usr/bin/env python3
"""Host-to-device copy rates on the box (clipgpu_test_h2d_bench): one SDMA copy, the pull kernel,
two SDMA copies, pull kernel beside SDMA (hipHostMalloc; and malloc + hipHostRegister); at the u8 bench batch's half (128 x 224 x 224 x 3 bytes) and
whole size.  One JSON line per (bytes, mode): µs and GB/s, median of REPS."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clip-embedder-rs_amd"))
from open_clip_inference import _lib  # noqa: E402

MODES = {0: "sdma", 1: "pull_kernel", 2: "two_sdma", 3: "pull_plus_sdma", 4: "sdma_registered",
         5: "pull_kernel_registered", 6: "two_sdma_registered"}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for nbytes in (128 * 224 * 224 * 3, 256 * 224 * 224 * 3):
        for mode, name in MODES.items():
            v = []
            for _ in range(reps):
                us = ctypes.c_double()
                _lib.check(_lib.lib().clipgpu_test_h2d_bench(nbytes, mode, 10, ctypes.byref(us)))
                v.append(us.value)
            m = statistics.median(v)
            print(json.dumps({"bytes": nbytes, "mode": name, "us_median": round(m, 1),
                              "GBps": round(nbytes / m / 1e3, 2), "us_all": [round(x, 1) for x in v]}), flush=True)


if __name__ == "__main__":
    main()
