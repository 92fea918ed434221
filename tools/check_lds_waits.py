#!/usr/bin/env python3
"""Static check of the inline-asm LDS fragment reads in the built GEMM kernels.

The pipelined GEMMs read their MFMA fragments with inline-asm `ds_read_b128` (gemm_util.hpp) and
retire them with an inline-asm `s_waitcnt lgkmcnt(0)` whose fake "+v" operands keep every consumer
below the wait.  The compiler believes an asm output is written AT the asm statement, so nothing
stops its register allocator from inserting spill code (a `scratch_store` of the destination, a
reload into it, a copy) between the asm read and the wait: the spill then stores the register
before the LDS data arrives, or the late LDS data overwrites what the compiler put there.  Either
is a timing-dependent race that no functional test is sure to see.

This scans the disassembly of every kernel for any instruction that names a vector register while
a `ds_read` into it may still be outstanding, over the kernel's control-flow graph (a forward
"may be pending" dataflow: lgkmcnt counts LDS operations in issue order, so `lgkmcnt(N)` retires
all but the N youngest; at a join the pending lists are merged youngest-aligned).

usage: check_lds_waits.py <disassembly.s | code object | .o/.so with a .hip_fatbin> [kernel-regex]
Prints the affected kernels; exit 1 when a hazard is found.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")
FUNC = re.compile(r"^([0-9a-f]+) <(.*)>:$")
ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
TARGET = re.compile(r"<[^>]*\+0x([0-9a-f]+)>")
MAXQ = 64


def regs(text):
    out = set()
    for kind, one, lo, hi in REG.findall(text):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return frozenset(out)


def disassemble(path):
    if path.endswith(".s"):
        return open(path).read()
    with tempfile.TemporaryDirectory() as d:
        co = path
        with open(path, "rb") as f:
            magic = f.read(4)
        if magic == b"\x7fELF":
            secs = subprocess.run([f"{LLVM}/llvm-objdump", "-h", path], capture_output=True, text=True).stdout
            if ".hip_fatbin" in secs:
                fb = os.path.join(d, "fatbin.bin")
                subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fb], check=True)
                co = os.path.join(d, "dev.co")
                subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={fb}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}", "--unbundle"],
                               check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], capture_output=True, text=True, check=True).stdout


def functions(asm):
    """{name: [(addr, instruction text)]}"""
    out, cur = {}, None
    for line in asm.splitlines():
        s = line.strip()
        m = FUNC.match(s)
        if m:
            cur = out.setdefault(m.group(2), [])
            base = int(m.group(1), 16)
            cur.append(("base", base))
            continue
        if cur is None or not s or s.startswith("//"):
            continue
        a = ADDR.search(s)
        ins = s.split("//")[0].strip()
        if ins.startswith("s_branch") or ins.startswith("s_cbranch"):
            t = TARGET.search(s)  # the target symbol is printed in the comment
            if t:
                ins += f" <+0x{t.group(1)}>"
        if a and ins:
            cur.append((int(a.group(1), 16), ins))
    return out


def merge(a, b):
    if a is None:
        return b
    n = max(len(a), len(b))
    pa = [frozenset()] * (n - len(a)) + list(a)
    pb = [frozenset()] * (n - len(b)) + list(b)
    return tuple(x | y for x, y in zip(pa, pb))


def step(state, ins, hazards=None, where=None):
    op = ins.split()[0]
    if op == "s_waitcnt":
        mm = re.search(r"lgkmcnt\((\d+)\)", ins)
        if mm:
            n = int(mm.group(1))
            state = state[len(state) - n:] if n else ()
        return state
    if op.startswith("s_"):
        if op.startswith("s_load") or op.startswith("s_buffer_load"):
            state = (state + (frozenset(),))[-MAXQ:]
        return state
    used = regs(ins)
    if hazards is not None:
        for p in state:
            if used & p:
                hazards.append(where)
                break
    if op.startswith("ds_read") or op.startswith("ds_load"):
        state = (state + (regs(ins.split(None, 1)[1].split(",")[0]),))[-MAXQ:]
    elif op.startswith("ds_") or op.startswith("flat_"):
        state = (state + (frozenset(),))[-MAXQ:]
    return state


def scan_function(name, body):
    base = body[0][1]
    ins = body[1:]
    if not ins:
        return []
    idx = {a: i for i, (a, _) in enumerate(ins)}
    leaders = {0}
    succ_of = {}
    for i, (a, t) in enumerate(ins):
        op = t.split()[0]
        if op.startswith("s_branch") or op.startswith("s_cbranch"):
            m = TARGET.search(t)
            tgt = idx.get(base + int(m.group(1), 16)) if m else None
            if tgt is not None:
                leaders.add(tgt)
            if i + 1 < len(ins):
                leaders.add(i + 1)
            succ_of[i] = ([tgt] if tgt is not None else []) + ([i + 1] if op.startswith("s_cbranch") and i + 1 < len(ins) else [])
        elif op in ("s_endpgm", "s_setpc_b64", "s_trap"):
            succ_of[i] = []
            if i + 1 < len(ins):
                leaders.add(i + 1)
    starts = sorted(leaders)
    blocks = []
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(ins)
        blocks.append((s, e))
    bidx = {s: k for k, (s, e) in enumerate(blocks)}
    succ = []
    for s, e in blocks:
        last = e - 1
        if last in succ_of:
            succ.append([bidx[x] for x in succ_of[last] if x in bidx])
        else:
            succ.append([bidx[e]] if e in bidx else [])
    entry = [None] * len(blocks)
    entry[0] = ()
    work = [0]
    while work:
        k = work.pop()
        st = entry[k]
        s, e = blocks[k]
        for i in range(s, e):
            st = step(st, ins[i][1])
        for n in succ[k]:
            m = merge(entry[n], st)
            if m != entry[n]:
                entry[n] = m
                work.append(n)
    hazards = []
    for k, (s, e) in enumerate(blocks):
        st = entry[k]
        if st is None:
            continue
        for i in range(s, e):
            st = step(st, ins[i][1], hazards, ins[i][1])
    return hazards


def scan(asm, kernel_re=None):
    out = {}
    for name, body in functions(asm).items():
        if kernel_re and not re.search(kernel_re, name):
            continue
        hz = scan_function(name, body)
        if hz:
            out[name] = hz
    return out


def main():
    if len(sys.argv) < 2:
        print(__doc__)
        return 2
    res = scan(disassemble(sys.argv[1]), sys.argv[2] if len(sys.argv) > 2 else None)
    for k, hz in sorted(res.items()):
        print(f"{k}: {len(hz)} use(s) of a possibly outstanding LDS read, e.g. {hz[0]}")
    print(f"{sum(len(v) for v in res.values())} hazards in {len(res)} kernels")
    return 1 if res else 0


if __name__ == "__main__":
    sys.exit(main())
