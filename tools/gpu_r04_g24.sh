#!/bin/bash
# Tile-order group A/B in the two-lane bench (CLIPGPU_TILE_GROUP 8 default / 1 / 4 / 16 library variants).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ROUNDS=2 VARIANTS="g8|;g1||g1;g4||g4;g16||g16" timeout -k 10 1000 bash tools/bench_variants.sh
echo done
