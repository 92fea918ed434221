#!/bin/bash
# Younger-half priority on the text leg too (vision + text bench; libclipgpu_noprio.so = without,
# libclipgpu_occ1.so = only on the one-block-per-CU 8-wave tiles 26 / 13).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BV_BASE="--no-cpu-baseline --no-fp8 --no-e2e --windows 3" ROUNDS=3 VARIANTS="prio|;noprio||noprio;occ1||occ1" timeout -k 10 1000 bash tools/bench_variants.sh
echo done
