# Ad-hoc GPU session: PYTEST_K selects tests of tests/test_gpu_api.py (-k expression), then
# STEPS_AFTER runs tools/gpu_check.sh steps.  Every GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 400 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_api.py} -k "$PYTEST_K" -x -v --timeout 150 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/t_sel.log 2>&1; rc=$?
  tail -15 gpurun_out/t_sel.log
  [ $rc -le 1 ] || exit $rc
fi
[ -z "${STEPS_AFTER:-}" ] || STEPS="$STEPS_AFTER" bash tools/gpu_check.sh
