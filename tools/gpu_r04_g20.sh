set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "w8_96x192 or 224x192_residual" -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_t27.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_t27.log; [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py::test_gemm_tile_choice_is_bit_exact -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_t27b.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_t27b.log; [ $rc -eq 0 ] || exit 1
VARIANTS="v_t|;v_27oc|--lanes 2 --tiles 18,27,15,27;v_27o|--lanes 2 --tiles 18,27,15,26;v_27c|--lanes 2 --tiles 18,26,15,27;v_27f|--lanes 2 --tiles 18,26,27,26" ROUNDS=2 bash tools/bench_variants.sh || exit $?
echo ALLDONE
