set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_SEL="tests/test_gpu_configs.py tests/test_gpu_api.py::test_tile_table_is_deterministic_and_bit_invisible" \
STEPS="tests_sel" bash tools/gpu_check.sh || exit $?
VARIANTS="v_t|;v_f17|--lanes 2 --tiles 18,26,17,26" ROUNDS=2 bash tools/bench_variants.sh || exit $?
echo ALLDONE
