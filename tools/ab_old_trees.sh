# Same-box A/B of the round-end trees (tools/ab_trees/rNN: bench.py + package + built library of
# each round's final commit, copied from `git archive`, gitignored) against this tree: the vision
# leg of each tree's own bench.py, interleaved, ROUNDS times.  One JSON line per run in
# gpurun_out/ab_trees.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
OUT=$PWD/gpurun_out/ab_trees.jsonl
for i in $(seq 1 "$ROUNDS"); do
  for t in cur r01 r02 r03; do
    if [ "$t" = cur ]; then d=.; extra="--no-e2e --windows 3"; else d=tools/ab_trees/$t; extra=""; fi
    [ "$t" = r01 ] || [ "$t" = cur ] || extra="$extra --no-e2e"
    echo "=== $t round $i $(date +%T)"
    (cd "$d" && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp8 --no-text $extra \
        > "$OLDPWD/gpurun_out/ab_${t}_$i.log" 2>&1) || { echo "ab $t failed rc=$?"; tail -5 "gpurun_out/ab_${t}_$i.log"; exit 1; }
    python3 - "$t" "$i" "gpurun_out/ab_${t}_$i.log" >> "$OUT" <<'PY' || exit 1
import json, sys
t, i, path = sys.argv[1:4]
line = [json.loads(l) for l in open(path) if l.startswith("{")][-1]
w = line.get("windows") or {}
print(json.dumps({"tree": t, "round": int(i), "value": line["value"], "ms_per_step": line["ms_per_step"],
                  "c_fc_us": (line.get("roofline") or {}).get("avg_launch_us"),
                  "gemm_tiles": line.get("gemm_tiles"), "sclk_mhz": line.get("sclk_mhz"),
                  "windows_median": w.get("median")}))
PY
    tail -1 "$OUT"
  done
done
