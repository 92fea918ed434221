#!/bin/bash
# Round-4 final tree: full GPU suite + smoke, then the bench, the vision kernel trace, the rocprofv3
# kernel-stats profile and the per-site PMC passes.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="tests smoke bench vtrace prof" bash tools/gpu_check.sh || exit $?
PMC_LABEL="round-4 final tree (r04_final)" STEPS="pmc" bash tools/gpu_check.sh || exit $?
echo ALLDONE
