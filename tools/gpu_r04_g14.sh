set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/bench_models.py lanesab > gpurun_out/lanesab.jsonl 2> gpurun_out/lanesab.err || { echo "lanesab rc=$?"; tail -5 gpurun_out/lanesab.err; exit 1; }
cat gpurun_out/lanesab.jsonl
BV_BASE="--no-cpu-baseline --no-fp8 --no-e2e --windows 0" \
VARIANTS="t_table|;t_26oc|--text-tiles 18,26,18,26;t_26c|--text-tiles 18,17,18,26;t_26o|--text-tiles 18,26,18,15" \
ROUNDS=2 bash tools/bench_variants.sh || exit $?
echo ALLDONE
