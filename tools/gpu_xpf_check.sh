#!/bin/bash
# GPU session for the residual prefetch (GemmParams::xpf, CLIPGPU_GEMM_XPF): bit-exactness + race
# check over every residual tile, the stamp timeline of the table tiles (baseline build), interleaved
# GEMM A/B with and without it at the residual trunk shapes, then whole-forward A/B of engines.
# Each GPU step has its own limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name (limit ${lim}s) $(date +%T)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc $(date +%T)"
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
step xpf_tests 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -rf -p no:cacheprovider -x \
    --timeout 300 --timeout-method thread -k "residual_prefetch or test_gemm_residual" || exit $?
if [ -f clip-embedder-rs_amd/lib/libclipgpu_stamps.so ]; then
  step stamps 300 python tools/gemm_stamps.py t17_ t18_ || exit $?
fi
for shp in ${SHAPES:-"12800 768 768 1 0" "12800 768 3072 1 0" "78848 512 2048 1 0" "46720 1280 5120 1 0"}; do
  set -- $shp
  step "xab_$1x$2x$3" 300 python tools/gemm_ab.py $1 $2 $3 $4 $5 ${TILES:-17,17x,13,13x,18,18x} 7 10 || exit $?
done
step eab_vision 300 python tools/engine_env_ab.py --workload b32_vision "" "CLIPGPU_GEMM_XPF=1" || exit $?
step eab_text 300 python tools/engine_env_ab.py --workload b32_text "" "CLIPGPU_GEMM_XPF=1" || exit $?
echo "=== done"
