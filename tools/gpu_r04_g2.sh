set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="tests" bash tools/gpu_check.sh || exit $?
AB_SPECS="12800 768 3072 1 0 17,26,28;12800 768 768 1 0 17,26,28;12544 768 3072 1 0 17,26,28;12800 2304 768 0 0 18,26,28" STEPS="ab" bash tools/gpu_check.sh || exit $?
STEPS="smoke bench" bash tools/gpu_check.sh || exit $?
PIN_TILES=18,26,18,26 STEPS="bench_pin" bash tools/gpu_check.sh || exit $?
PIN_TILES=18,28,18,28 STEPS="bench_pin" bash tools/gpu_check.sh || exit $?
echo ALLDONE
