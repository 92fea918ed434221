#!/usr/bin/env python3
"""Register / LDS / spill usage of the GEMM kernels in a built object or library.

usage: kernel_regs.py <.o | .so with a .hip_fatbin> [kernel-regex]
Reads the code object's AMDGPU metadata note (llvm-readelf --notes) and prints, per kernel,
vgpr / agpr counts, spills, LDS bytes and the demangled name.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(path, d):
    fb = os.path.join(d, "fatbin.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fb], check=True)
    co = os.path.join(d, "dev.co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}", "--unbundle"], check=True)
    return co


def short(mangled):
    """gemm_pipe_kernel<bf16,256,256,2,4,...> from the Itanium name (the image's c++filt predates
    the DF16b mangling)."""
    m = re.search(r"N_1\d+(\w+?)I(.*)EEvN", mangled)
    if not m:
        return mangled
    base, args = m.groups()
    args = args.replace("DF16b", "bf16,").replace("DF16_", "f16,")
    args = re.sub(r"Li(-?\d+)E", r"\1,", args).rstrip(",")
    return f"{base}<{args}>"


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    with tempfile.TemporaryDirectory() as d:
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", code_object(path, d)],
                               capture_output=True, text=True).stdout
    rows, cur = [], {}
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s*(.*)$", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "agpr_count":  # first key of each kernel's record
            cur = {"agpr": v}
            rows.append(cur)
        elif k in ("group_segment_fixed_size", "vgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                   "private_segment_fixed_size", "name"):
            cur[k] = v
    for r in rows:
        n = short(r.get("name", ""))
        if pat.search(n):
            print(f"vgpr {r.get('vgpr_count', '?'):>3} agpr {r.get('agpr', '?'):>3} "
                  f"spill {r.get('vgpr_spill_count', '?'):>2} scratch {r.get('private_segment_fixed_size', '?'):>4} "
                  f"lds {r.get('group_segment_fixed_size', '?'):>6}  {n[:200]}")


if __name__ == "__main__":
    main()
