#!/bin/bash
# Per-site tile order (qkv / c_proj walk N first): parity subset, same-box A/B against the uniform
# order (libclipgpu_g8site.so), then the bench + per-site PMC passes of the new default.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEPS=tests_sel PYTEST_SEL="tests/test_gpu_parity.py tests/test_gpu_api.py" bash tools/gpu_check.sh
ROUNDS=3 VARIANTS="site|;uniform||g8site" timeout -k 10 900 bash tools/bench_variants.sh
PMC_LABEL="round-4 run r04_g25 (per-site tile order)" STEPS="bench pmc" bash tools/gpu_check.sh
echo done
