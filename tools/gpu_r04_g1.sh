set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_SEL="tests/test_gpu_kernels.py::test_224x192_residual_tile_is_bit_exact tests/test_gpu_bench_config.py::test_device_entry_is_ordered_on_the_callers_stream" \
STEPS="tests_sel" bash tools/gpu_check.sh || exit $?
AB_SPECS="12800 768 3072 1 0 17,26,27;12800 768 768 1 0 17,26,27;12544 768 3072 1 0 17,26,27;39424 512 2048 1 0 15,17,26" STEPS="ab" bash tools/gpu_check.sh || exit $?
STEPS="bench" bash tools/gpu_check.sh || exit $?
PIN_TILES=18,26,18,26 STEPS="bench_pin" bash tools/gpu_check.sh || exit $?
PIN_TILES=18,27,18,27 STEPS="bench_pin" bash tools/gpu_check.sh || exit $?
PIN_TILES=18,17,18,17 STEPS="bench_pin" bash tools/gpu_check.sh || exit $?
echo ALLDONE
