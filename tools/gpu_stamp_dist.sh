set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local n=$1 l=$2; shift 2; echo "=== $n"; timeout -k 10 $l "$@" > gpurun_out/$n.log 2>&1; local rc=$?; cat gpurun_out/$n.log | grep -v amdgpu.ids; return $rc; }
run dist_out17 120 python tools/gemm_stamp_dist.py 12800 768 768 1 0 17 2 || exit $?
run dist_cfc18 120 python tools/gemm_stamp_dist.py 12800 3072 768 0 1 18 1 || exit $?
run dist_qkv18 120 python tools/gemm_stamp_dist.py 12800 2304 768 0 0 18 1 || exit $?
run dist_out9 120 python tools/gemm_stamp_dist.py 12800 768 768 1 0 9 1 || exit $?
run dist_out7 120 python tools/gemm_stamp_dist.py 12800 768 768 1 0 7 1 || exit $?
run dist_out13 120 python tools/gemm_stamp_dist.py 12800 768 768 1 0 13 1 || exit $?
run eab 200 python tools/engine_env_ab.py --workload b32_vision --rounds 5 "" "CLIPGPU_LANES=2" || exit $?
