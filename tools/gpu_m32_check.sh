#!/bin/bash
# GPU session for the 32x32x16-MFMA tiles (gemm_pipe_kernel M32 = 1, tiles 21-25): kernel numerics and
# bit-exactness tests, the LDS-poison race check, the whole-tower tile-pin bit-exactness test, then
# interleaved A/B timings at the trunk shapes.  Each GPU step has its own limit; a failure ends it.
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
step m32_kernels 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -rf -p no:cacheprovider -x \
    --timeout 300 --timeout-method thread -k "m32 or never_read_a_stage or half_tile" || exit $?
for shp in ${SHAPES:-"12800 3072 768 0 1" "12800 2304 768 0 0" "12800 768 3072 1 0" "12800 768 768 1 0" "6400 3072 768 0 1" "78848 2048 512 0 1" "78848 512 2048 1 0"}; do
  set -- $shp
  step "ab_$1x$2x$3" 300 python tools/gemm_ab.py $1 $2 $3 $4 $5 ${TILES:-18,21,17,22,23,24,25} 5 10 || exit $?
done
step m32_pins 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf -p no:cacheprovider -x \
    --timeout 300 --timeout-method thread -k "tile_choice" || exit $?
echo "=== done"
