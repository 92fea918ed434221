# Interleaved same-box A/B of bench.py variants.  VARIANTS: ';'-separated "label|extra bench
# args[|library]" (library: a lib/libclipgpu_<name>.so variant, `make variant`, via CLIPGPU_LIB); ROUNDS rounds; BV_BASE replaces the default base args (vision leg only).  One JSON summary line per run in
# gpurun_out/bench_variants.jsonl (value, ms/step, c_fc launch, tiles, lanes, clock under load).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
OUT=gpurun_out/bench_variants.jsonl
IFS=';' read -ra VS <<< "${VARIANTS}"
for i in $(seq 1 "$ROUNDS"); do
  for v in "${VS[@]}"; do
    label=${v%%|*}; extra=${v#*|}; vlib=
    if [[ "$extra" == *"|"* ]]; then vlib=${extra#*|}; extra=${extra%%|*}; fi
    if [ -n "$vlib" ]; then export CLIPGPU_LIB=$PWD/clip-embedder-rs_amd/lib/libclipgpu_$vlib.so; else unset CLIPGPU_LIB; fi
    log="gpurun_out/bv_${label}_$i.log"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BV_BASE:---no-cpu-baseline --no-fp8 --no-text --no-e2e --windows 3} \
        $extra > "$log" 2>&1 || { echo "variant $label failed rc=$?"; tail -5 "$log"; exit 1; }
    python3 - "$label" "$i" "$log" >> "$OUT" <<'PY' || exit 1
import json, sys
label, i, path = sys.argv[1:4]
l = [json.loads(x) for x in open(path) if x.startswith("{")][-1]
w = l.get("windows") or {}
print(json.dumps({"variant": label, "round": int(i), "value": l["value"], "windows_median": w.get("median"),
                  "ms_per_step": l["ms_per_step"], "c_fc_us": l["roofline"]["avg_launch_us"],
                  "tiles": l.get("gemm_tiles_env"), "lanes": l.get("lanes_env"), "sclk_mhz": l.get("sclk_mhz"),
                  "whole_frac": l.get("whole_forward_frac_of_peak"),
                  "text_value": (l.get("text") or {}).get("value"), "text_lanes": (l.get("text") or {}).get("lanes")}))
PY
    tail -1 "$OUT"
  done
done
