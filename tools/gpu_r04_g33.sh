#!/bin/bash
# Static younger-half priority in the MX-fp8 GEMM (libclipgpu_mxpr.so) on the fp8 vision leg; the
# shipped bf16 tree (GEMM younger-half priority on) once more against itself for the noise floor.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ROUNDS=3 VARIANTS="fp8|--dtype fp8;fp8pr|--dtype fp8|mxpr;bf16|" timeout -k 10 900 bash tools/bench_variants.sh
echo done
