#!/bin/bash
# Host-to-device copy rates (tools/h2d_bench.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/h2d_bench.py 5 > gpurun_out/h2d_bench.jsonl 2> gpurun_out/h2d_bench.err
echo done
