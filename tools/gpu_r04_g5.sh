set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/host_plan_ab.py 3 8 > gpurun_out/host_plan_ab.jsonl 2> gpurun_out/host_plan_ab.err || { echo "host plan rc=$?"; tail -5 gpurun_out/host_plan_ab.err; exit 1; }
cat gpurun_out/host_plan_ab.jsonl
VARIANTS="l1_table|;l2_table|--lanes 2;l2_15|--lanes 2 --tiles 15,15,15,15;l2_15_17|--lanes 2 --tiles 15,17,15,17;l2_14_17|--lanes 2 --tiles 14,17,15,17;l2_3_15|--lanes 2 --tiles 3,15,15,15" \
ROUNDS=2 bash tools/bench_variants.sh || exit $?
echo ALLDONE
