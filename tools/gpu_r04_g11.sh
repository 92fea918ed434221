set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="v_l2|;v_26oc|--lanes 2 --tiles 18,26,15,26;v_26o|--lanes 2 --tiles 18,26,15,15;v_13q|--lanes 2 --tiles 13,15,15,15;v_14_26oc|--lanes 2 --tiles 14,26,15,26" ROUNDS=3 bash tools/bench_variants.sh || exit $?
echo ALLDONE
