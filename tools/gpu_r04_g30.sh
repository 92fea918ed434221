#!/bin/bash
# Host path: registered inputs' H2Ds queued before the first forward (default, copy_stream 1) vs
# interleaved with the forwards (5); registered-buffer parity tests first.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEPS=tests_sel PYTEST_SEL="tests/test_gpu_parity.py::test_registered_host_buffers_are_bit_exact" bash tools/gpu_check.sh
HP_MODES=1,5 timeout -k 10 400 python -u tools/host_plan_ab.py 4 8 > gpurun_out/host_copies_first.jsonl 2> gpurun_out/host_copies_first.err
echo done
