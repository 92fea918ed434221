#!/bin/bash
# One GPU session: kernel + parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / timeout (exit >= 2 for pytest,
# != 0 for the others) ends the script.  Output goes to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests bench prof}
run() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name (limit ${lim}s) $(date +%T)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc $(date +%T)"
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
for s in $STEPS; do
  case $s in
    tests)
      run pytest_gpu 900 python -m pytest tests -m gpu -q -rf -p no:cacheprovider
      rc=$?; [ $rc -le 1 ] || exit $rc ;;
    sweep)
      run gemm_sweep 600 python tools/gemm_sweep.py || exit $? ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
      run bench 600 python bench.py --steps 20 --warmup 5 || exit $? ;;
    prof)
      run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
          python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit $?
      find gpurun_out/prof -name "*kernel_stats.csv" | head -3 ;;
  esac
done
echo "=== done"
