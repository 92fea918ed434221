#!/bin/bash
# Wave priority in the GEMM K-loop (guide T5): 1 = static s_setprio 1 for the younger half of
# 8-wave blocks, 2 = s_setprio 1 around each phase's MFMA groups; two-lane bench A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ROUNDS=3 VARIANTS="base|;pr1||pr1;pr2||pr2" timeout -k 10 900 bash tools/bench_variants.sh
echo done
