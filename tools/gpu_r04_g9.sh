set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BV_BASE="--no-cpu-baseline --no-fp8 --no-e2e --windows 0" \
VARIANTS="t_table|;t_18_15_18_15|--text-tiles 18,15,18,15;t_18_15_15_15|--text-tiles 18,15,15,15;t_14_15_15_15|--text-tiles 14,15,15,15;t_18_17_15_15|--text-tiles 18,17,15,15" \
ROUNDS=2 bash tools/bench_variants.sh || exit $?
mv gpurun_out/bench_variants.jsonl gpurun_out/bench_variants_text.jsonl
VARIANTS="v_l2|;v_l3|--lanes 3 --tiles 18,15,15,15;v_l4|--lanes 4 --tiles 18,15,15,15" ROUNDS=2 bash tools/bench_variants.sh || exit $?
echo ALLDONE
