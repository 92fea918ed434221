#!/bin/bash
# Tile-order group A/B (CLIPGPU_TILE_GROUP 1 / 4 / 8 (default) / 16): per-site standalone launches
# (tools/ld_pad_ab.py, pitch 0 column) and the interleaved two-lane bench; FETCH_SIZE of c_proj per group.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/clip-embedder-rs_amd/lib
for g in 8 1 4 16; do
  lib=$L/libclipgpu_g$g.so; [ $g = 8 ] && lib=$L/libclipgpu.so
  CLIPGPU_LIB=$lib timeout -k 10 200 python -u tools/ld_pad_ab.py 3 > gpurun_out/group_g$g.jsonl 2>&1
  CLIPGPU_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/grpmc_f$g -o run -- python3 tools/ld_pad_ab.py one c_proj 0 10 > gpurun_out/grpmc_f$g.log 2>&1
done
ROUNDS=2 VARIANTS="g8|;g1||g1;g4||g4;g16||g16" timeout -k 10 1000 tools/bench_variants.sh
echo done
