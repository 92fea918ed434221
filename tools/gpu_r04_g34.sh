#!/bin/bash
# Priority 1 for odd blocks of the 4-wave GEMM tiles (c_fc's tile 15 pairs two blocks per CU):
# two-lane bench A/B (libclipgpu_obp.so).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ROUNDS=3 VARIANTS="base|;obp||obp" timeout -k 10 900 bash tools/bench_variants.sh
echo done
