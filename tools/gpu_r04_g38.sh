#!/bin/bash
# Last check of the committed library: API tests + smoke.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_SEL="tests/test_gpu_api.py tests/test_gpu_parity.py" STEPS="tests_sel smoke" bash tools/gpu_check.sh || exit $?
echo ALLDONE
