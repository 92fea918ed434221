set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_SEL="tests/test_gpu_api.py::test_tile_table_is_deterministic_and_bit_invisible tests/test_gpu_bench_config.py" \
STEPS="tests_sel" bash tools/gpu_check.sh || exit $?
STEPS="bench vtrace pmc" bash tools/gpu_check.sh || exit $?
VARIANTS="v_t|;v_f18|--lanes 2 --tiles 18,26,18,26;v_f13|--lanes 2 --tiles 18,26,13,26;v_f2|--lanes 2 --tiles 18,26,2,26" ROUNDS=2 bash tools/bench_variants.sh || exit $?
echo ALLDONE
