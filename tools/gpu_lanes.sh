#!/bin/bash
# Bench the vision/text legs at 1..4 concurrent lanes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for L in 1 2 3 4; do
  CLIPGPU_LANES=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lanes_$L.log 2>&1 || exit $?
  echo "lanes=$L"; grep '^{' gpurun_out/lanes_$L.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['gemm_tiles'], d['roofline']['avg_launch_us'], d['text']['value'])"
done
