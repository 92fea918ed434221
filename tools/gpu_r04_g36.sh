#!/bin/bash
# Tile table re-check with the younger-half priority on (vision two lanes): c_fc on the 8-wave tiles
# 18 / 26 (which now carry the priority) and qkv on 14, against the table (18,26,15,26).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ROUNDS=2 VARIANTS="t|;f18|--tiles 18,26,18,26;f26|--tiles 18,26,26,26;q14|--tiles 14,26,15,26" timeout -k 10 1000 bash tools/bench_variants.sh
echo done
