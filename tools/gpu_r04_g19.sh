set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="v_p0|;v_p1|--lane-priority 1;v_p2|--lane-priority 2" ROUNDS=3 bash tools/bench_variants.sh || exit $?
echo ALLDONE
