#!/bin/bash
# A/B of engine settings in one GPU session: bench.py (vision leg, breakdown) once per setting,
# alternating rounds.  usage: ROUNDS=2 bash tools/bench_ab.sh "CLIPGPU_LANES=2" "CLIPGPU_LANES=1"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 "${ROUNDS:-2}"); do
  i=0
  for setting in "$@"; do
    log=gpurun_out/ab_${r}_${i}.log
    env $setting timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp8 --no-e2e \
        ${BENCH_ARGS:---no-text --breakdown} > $log 2>&1 || { tail -5 $log; exit 1; }
    python3 tools/bench_summary.py "$setting" $log
    i=$((i+1))
  done
done
