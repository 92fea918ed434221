#!/bin/bash
# 4-wave residual tiles 29 (96x192) / 30 (128x192, 2 x 80 KiB per CU): bit-exactness, standalone
# out_proj / c_proj, then the two-lane bench with them at out_proj / c_proj (patch stays 26).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEPS=tests_sel PYTEST_SEL="tests/test_gpu_kernels.py" bash tools/gpu_check.sh
timeout -k 10 300 python3 tools/gemm_ab.py 6400 768 3072 1 0 26,29,30,15 5 20 > gpurun_out/res_ab.log 2>&1
timeout -k 10 300 python3 tools/gemm_ab.py 6400 768 768 1 0 26,29,30,15 5 20 >> gpurun_out/res_ab.log 2>&1
cat gpurun_out/res_ab.log
ROUNDS=2 VARIANTS="t26|;t29|--tiles 18,29,15,29;t30|--tiles 18,30,15,30;t30c|--tiles 18,26,15,30" timeout -k 10 900 bash tools/bench_variants.sh
echo done
