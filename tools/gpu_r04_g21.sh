#!/bin/bash
# Row-pitch A/B of the trunk GEMMs (tools/ld_pad_ab.py) + FETCH_SIZE of c_proj at pitch 3072 / 3136.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ld_pad_ab.py 5 > gpurun_out/ld_pad_ab.jsonl 2> gpurun_out/ld_pad_ab.err
for pad in 0 64; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ldpmc_f$pad -o run -- python3 tools/ld_pad_ab.py one c_proj $pad 10 > gpurun_out/ldpmc_f$pad.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/ldpmc_w$pad -o run -- python3 tools/ld_pad_ab.py one c_proj $pad 10 > gpurun_out/ldpmc_w$pad.log 2>&1
done
echo done
