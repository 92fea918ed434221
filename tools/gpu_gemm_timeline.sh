#!/bin/bash
# GPU session after a GEMM schedule change: bit-exactness / race-check kernel tests, the per-block
# launch timeline of the table tiles (stamp build), interleaved A/B of the table tiles at the trunk
# shapes, and the vision forward.  Each GPU step has its own limit; a failure ends the script.
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
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 40
  return $rc
}
step kt 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -rf -p no:cacheprovider -x \
    --timeout 300 --timeout-method thread -k "never_read_a_stage or half_tile or test_gemm_residual or three_stage" || exit $?
step pins 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf -p no:cacheprovider -x \
    --timeout 300 --timeout-method thread -k "tile_choice or tile_table" || exit $?
if [ -f clip-embedder-rs_amd/lib/libclipgpu_stamps.so ]; then
  step tl_out17 120 python tools/gemm_stamp_dist.py 12800 768 768 1 0 17 2 || exit $?
  step tl_cproj17 120 python tools/gemm_stamp_dist.py 12800 768 3072 1 0 17 2 || exit $?
  step tl_cfc18 120 python tools/gemm_stamp_dist.py 12800 3072 768 0 1 18 1 || exit $?
  step tl_qkv18 120 python tools/gemm_stamp_dist.py 12800 2304 768 0 0 18 1 || exit $?
fi
for shp in "12800 2304 768 0 0 18" "12800 3072 768 0 1 18" "12800 768 3072 1 0 17" "12800 768 768 1 0 17"; do
  set -- $shp
  step "ab_$1x$2x$3" 300 python tools/gemm_ab.py $1 $2 $3 $4 $5 $6 7 10 || exit $?
done
step bench_vision 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp8 --no-e2e --no-text || exit $?
echo "=== done"
