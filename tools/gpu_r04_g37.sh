#!/bin/bash
# Attention: the Q fragments loaded before the K / V staging when every wave owns one query tile
# (libclipgpu_qearly.so): attention tests on that library, then the two-lane bench A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CLIPGPU_LIB=$PWD/clip-embedder-rs_amd/lib/libclipgpu_qearly.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -k attention -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/qearly_tests.log 2>&1
tail -2 gpurun_out/qearly_tests.log
timeout -k 10 200 python3 tools/attn_bench.py > gpurun_out/attn_base.log 2>&1 || true
CLIPGPU_LIB=$PWD/clip-embedder-rs_amd/lib/libclipgpu_qearly.so timeout -k 10 200 python3 tools/attn_bench.py > gpurun_out/attn_qearly.log 2>&1 || true
ROUNDS=3 VARIANTS="base|;qearly||qearly" timeout -k 10 900 bash tools/bench_variants.sh
echo done
