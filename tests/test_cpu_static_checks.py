"""Static checks of the built GEMM code objects (CPU only: disassembly, no GPU).

The pipelined GEMMs read MFMA fragments with inline-asm ds_read_b128 and retire them with an
inline-asm lgkmcnt wait; nothing stops the register allocator from touching a destination register
(a spill store, a copy) between the two, which reads the register before the LDS data arrives.
tools/check_lds_waits.py scans every kernel's control-flow graph for such a use.  Round 3 found
exactly this in the race-check build of a dropped 224x256 tile (its extra instrumentation pushed
the kernel to 224 spilled registers), so the check runs on the product library AND
on the race-check library whose verdicts the GPU tests trust.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "clip-embedder-rs_amd", "lib")


@pytest.mark.parametrize("name", ["libclipgpu.so", "libclipgpu_poison.so"])
def test_no_fragment_register_is_used_before_its_lds_read_lands(name):
    path = os.path.join(LIBDIR, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not built")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_lds_waits.py"), path],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "0 hazards" in r.stdout, r.stdout[-2000:]
