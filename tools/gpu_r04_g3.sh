set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_SEL="tests/test_gpu_parity.py::test_registered_host_buffers_are_bit_exact tests/test_gpu_kernels.py::test_224x192_residual_tile_is_bit_exact tests/test_gpu_parity.py::test_gemm_tile_choice_is_bit_exact" \
STEPS="tests_sel" bash tools/gpu_check.sh || exit $?
STEPS="bench" bash tools/gpu_check.sh || exit $?
echo ALLDONE
