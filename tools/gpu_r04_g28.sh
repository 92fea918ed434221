#!/bin/bash
# Timeline of the registered u8 host path (tools/host_trace.py), kernel trace only (the memory-copy
# trace serialised the copies with the kernels: calls of 8.1 ms, 3.7 ms unprofiled).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/htrace2 -o run -- python3 tools/host_trace.py 8 > gpurun_out/htrace2.log 2>&1
python3 tools/host_trace.py analyze gpurun_out/htrace2 > gpurun_out/htrace_summary.txt
echo done
