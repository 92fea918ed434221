#!/bin/bash
# Residual-epilogue x-ring depth A/B for the 224x192 tile (26): x row blocks in flight per wave 3
# (default) / 4 / 5 / all 7 (14 spilled registers): standalone out_proj / c_proj, then the bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/clip-embedder-rs_amd/lib
for v in base xr4 xr5 xall; do
  lib=$L/libclipgpu_$v.so; [ $v = base ] && lib=$L/libclipgpu.so
  LD_PADS=0 CLIPGPU_LIB=$lib timeout -k 10 200 python -u tools/ld_pad_ab.py 5 out_proj c_proj > gpurun_out/xring_$v.jsonl 2>&1
done
ROUNDS=2 VARIANTS="base|;xr4||xr4;xr5||xr5;xall||xall" timeout -k 10 900 bash tools/bench_variants.sh
echo done
