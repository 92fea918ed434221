#!/bin/bash
# GPU session for the LayerNorm grid knob (CLIPGPU_LN_BLOCKS): numerics with multi-row waves, bits
# of the whole forward against the default grid, and interleaved bench A/B of grid caps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CLIPGPU_LN_BLOCKS=7 timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider -k layernorm \
    > gpurun_out/ln_tests.log 2>&1 || { tail -20 gpurun_out/ln_tests.log; exit 1; }
tail -1 gpurun_out/ln_tests.log
for w in b32_vision b32_text; do
  WORKLOAD=$w timeout -k 10 120 python tools/embed_bits.py gpurun_out/ln_default_$w.npy > /dev/null 2>&1 || exit 1
  for c in 1600 800 64; do
    WORKLOAD=$w CLIPGPU_LN_BLOCKS=$c timeout -k 10 120 python tools/embed_bits.py gpurun_out/ln_${c}_${w}.npy > /dev/null 2>&1 || exit 1
    echo -n "$w LN_BLOCKS=$c vs default: "; python tools/embed_bits.py --cmp gpurun_out/ln_default_$w.npy gpurun_out/ln_${c}_${w}.npy
  done
done
ROUNDS=${ROUNDS:-3} timeout -k 10 900 bash tools/bench_ab.sh "CLIPGPU_LN_BLOCKS=0" "CLIPGPU_LN_BLOCKS=2048" "CLIPGPU_LN_BLOCKS=1600" "CLIPGPU_LN_BLOCKS=800" || exit 1
echo "=== done"
