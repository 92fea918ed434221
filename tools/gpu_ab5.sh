# Round-5 session: residual-storage parity tests, then the interleaved A/B of residual storage and lane offset.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "residual" -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/t_resid.log 2>&1; rc=$?
tail -8 gpurun_out/t_resid.log
[ $rc -le 1 ] || exit $rc
ROUNDS=${ROUNDS:-2} BV_BASE="--no-cpu-baseline --no-fp8 --no-e2e --windows 2" VARIANTS="${VARIANTS}" \
    timeout -k 10 1000 bash tools/bench_variants.sh
