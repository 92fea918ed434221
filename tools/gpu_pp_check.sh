#!/bin/bash
# One GPU session for the ping-pong GEMM (gemm_pp.hip, tiles 19 / 20): kernel numerics + bit-exactness
# tests, the LDS-poison race check, interleaved A/B timings at the trunk shapes, and (DIAG=1) the
# 224x256 poison diagnosis variants.  Each GPU step has its own limit; a failure ends the script.
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
  tail -n 30 "gpurun_out/$name.log"
  return $rc
}
step pp_kernels 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -rf -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "pp_256 or pp_192 or never_read_a_stage" || exit $?
if [ "${DIAG:-0}" = 1 ]; then
  CLIPGPU_POISON_LIB=clip-embedder-rs_amd/lib/libclipgpu_diag224p.so CLIPGPU_REF_LIB=clip-embedder-rs_amd/lib/libclipgpu_diag224.so \
    step poison224 300 python tools/poison_diag.py 99,98,97 "12800,768,768,2;2000,3072,768,2;1000,600,256,2" 3 || exit $?
fi
for shp in "12800 3072 768 0 1" "12800 2304 768 0 0" "12800 768 3072 1 0" "12800 768 768 1 0" "78848 2048 512 0 1" "78848 512 2048 1 0" "46720 5120 1280 0 2" "46720 1280 5120 1 0"; do
  set -- $shp
  step "ab_$1x$2x$3" 300 python tools/gemm_ab.py $1 $2 $3 $4 $5 ${TILES:-3,14,18,19,13,17,20} 5 10 || exit $?
done
echo "=== done"
