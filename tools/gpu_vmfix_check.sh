#!/bin/bash
# GPU session after the "retire the LDS-DMA before the epilogue stores" fix: the LDS-poison race
# check over every pipelined tile (incl. the ping-pong tiles), the dropped 224x256 f32-store tile
# through its diagnostic poison build (failed massively before the fix), the GEMM kernel tests,
# interleaved A/B of the trunk shapes (the cost of the earlier wait), then the bench.
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
  tail -n 12 "gpurun_out/$name.log"
  return $rc
}
step mfma_probe 120 tools/bin/mfma_order_probe || exit $?
CLIPGPU_POISON_LIB=clip-embedder-rs_amd/lib/libclipgpu_diag224p.so CLIPGPU_REF_LIB=clip-embedder-rs_amd/lib/libclipgpu_diag224.so \
  step poison224_fixed 300 python tools/poison_diag.py 99 "12800,768,768,2;2000,3072,768,2;1000,600,256,2;12800,768,768,1" 3 || exit $?
step gemm_kernels 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py -m gpu -q -rf -p no:cacheprovider \
    --timeout 300 --timeout-method thread || exit $?
for shp in "12800 3072 768 0 1" "12800 2304 768 0 0" "12800 768 3072 1 0" "12800 768 768 1 0" "12544 768 3072 1 0"; do
  set -- $shp
  step "ab_$1x$2x$3" 300 python tools/gemm_ab.py $1 $2 $3 $4 $5 ${TILES:-14,17,18,19,20} 5 10 || exit $?
done
step bench 600 python bench.py --steps 20 --warmup 5 || exit $?
echo "=== done"
