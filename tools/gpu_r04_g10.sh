set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="v_l2|;v_26o|--lanes 2 --tiles 18,26,15,15;v_26c|--lanes 2 --tiles 18,15,15,26;v_26oc|--lanes 2 --tiles 18,26,15,26;v_26f|--lanes 2 --tiles 18,15,26,15;v_13c|--lanes 2 --tiles 18,15,15,13" ROUNDS=2 bash tools/bench_variants.sh || exit $?
echo ALLDONE
