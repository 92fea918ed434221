#!/usr/bin/env python3
"""One line per bench.py JSON log: value, tiles, serialized per-class ms (if --breakdown)."""
import json
import sys

label, path = sys.argv[1], sys.argv[2]
line = [json.loads(x) for x in open(path) if x.startswith("{")][-1]
bd = {k: v["ms_per_step"] for k, v in (line.get("breakdown_serialized") or {}).items()}
txt = line.get("text") or {}
print(f"{label:40s} {line['value']:9.1f} img/s  text {txt.get('value', '-')}  tiles {line['gemm_tiles_env']}  "
      f"c_fc {line['roofline']['avg_launch_us']}us  {bd}", flush=True)
