set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="tests smoke bench vtrace pmc" bash tools/gpu_check.sh || exit $?
timeout -k 10 420 python3 tools/mx_layer_sweep.py h14_text > gpurun_out/mx_layer_h14_text.jsonl 2> gpurun_out/mx_layer_h14_text.err || { echo "sweep rc=$?"; tail -5 gpurun_out/mx_layer_h14_text.err; exit 1; }
tail -3 gpurun_out/mx_layer_h14_text.jsonl
echo ALLDONE
