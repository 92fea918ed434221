#!/bin/bash
# Text tower: younger-half priority only at its 256x256 half-tile sites (qkv, c_fc; libclipgpu_tp18.so)
# against none (the shipped text setting); vision + text bench, 3 rounds.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BV_BASE="--no-cpu-baseline --no-fp8 --no-e2e --windows 3" ROUNDS=3 VARIANTS="base|;tp18||tp18" timeout -k 10 1000 bash tools/bench_variants.sh
echo done
