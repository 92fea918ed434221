#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the standalone c_proj launch (tile 26, 6400 rows) at pitch 3072 / 3136.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for pad in 0 64; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ldpmc_f$pad -o run -- python3 tools/ld_pad_ab.py one c_proj $pad 10 > gpurun_out/ldpmc_f$pad.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ldpmc_w$pad -o run -- python3 tools/ld_pad_ab.py one c_proj $pad 10 > gpurun_out/ldpmc_w$pad.log 2>&1
done
echo done
