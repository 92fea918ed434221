set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="bench vtrace pmc" bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python3 tools/host_plan_ab.py 3 8 > gpurun_out/host_plan_ab3.jsonl 2> gpurun_out/host_plan_ab3.err || { echo "host plan rc=$?"; tail -5 gpurun_out/host_plan_ab3.err; exit 1; }
cat gpurun_out/host_plan_ab3.jsonl
timeout -k 10 420 python3 tools/mx_layer_sweep.py h14_text > gpurun_out/mx_layer_h14_text.jsonl 2> gpurun_out/mx_layer_h14_text.err || { echo "sweep rc=$?"; tail -5 gpurun_out/mx_layer_h14_text.err; exit 1; }
tail -3 gpurun_out/mx_layer_h14_text.jsonl
echo ALLDONE
