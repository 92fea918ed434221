set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="tests smoke bench" bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python bench.py --gather --steps 10 --warmup 3 --no-cpu-baseline --no-fp8 --no-e2e > gpurun_out/bench_gather.log 2>&1 || { echo "gather rc=$?"; tail -5 gpurun_out/bench_gather.log; exit 1; }
tail -1 gpurun_out/bench_gather.log | head -c 600
echo ALLDONE
