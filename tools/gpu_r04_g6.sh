set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_SEL="tests/test_gpu_parity.py::test_text_parity tests/test_gpu_parity.py::test_last_layer_pruning_is_bit_exact tests/test_gpu_parity.py::test_siglip2_text_is_not_trimmed_and_pools_the_last_position tests/test_gpu_parity.py::test_registered_host_buffers_are_bit_exact tests/test_gpu_configs.py::test_so400m_siglip2_text_shard_128" \
STEPS="tests_sel" bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python3 tools/host_plan_ab.py 3 8 > gpurun_out/host_plan_ab2.jsonl 2> gpurun_out/host_plan_ab2.err || { echo "host plan rc=$?"; tail -5 gpurun_out/host_plan_ab2.err; exit 1; }
cat gpurun_out/host_plan_ab2.jsonl
VARIANTS="l2_3_15|--lanes 2 --tiles 3,15,15,15;l2_14_15|--lanes 2 --tiles 14,15,15,15;l2_18_15|--lanes 2 --tiles 18,15,15,15;l2_3_15_3|--lanes 2 --tiles 3,15,3,15;l2_3_15_14|--lanes 2 --tiles 3,15,14,15;l2_2_15|--lanes 2 --tiles 2,15,15,15;l2_3_1|--lanes 2 --tiles 3,1,15,15" \
ROUNDS=2 bash tools/bench_variants.sh || exit $?
echo ALLDONE
