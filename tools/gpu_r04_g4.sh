set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_SEL="tests/test_gpu_parity.py::test_registered_host_buffers_are_bit_exact tests/test_gpu_parity.py::test_vision_chunking_and_order tests/test_gpu_parity.py::test_vision_u8_path_matches_f32_path tests/test_gpu_parity.py::test_graph_replay_reads_fresh_inputs_and_matches_direct_launches" \
STEPS="tests_sel" bash tools/gpu_check.sh || exit $?
STEPS="bench" bash tools/gpu_check.sh || exit $?
bash tools/ab_old_trees.sh || exit $?
timeout -k 10 480 python3 tools/mx_layer_sweep.py b32_text > gpurun_out/mx_layer_b32_text.jsonl 2> gpurun_out/mx_layer_b32_text.err || { echo "sweep rc=$?"; tail -5 gpurun_out/mx_layer_b32_text.err; exit 1; }
tail -3 gpurun_out/mx_layer_b32_text.jsonl
echo ALLDONE
