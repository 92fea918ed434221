#!/bin/bash
# One GPU session, parameterised by STEPS (the steps below, in order; e.g.
#   STEPS="bench_quick ablate" bash tools/gpu_check.sh
# ): kernel + parity tests, smoke, bench, rocprofv3 kernel-trace summary, PMC passes, A/B runs.
# Every GPU step has its own time limit; a crash / timeout (exit >= 2 for pytest,
# != 0 for the others) ends the script.  Output goes to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# steps: tests, tests_sel (PYTEST_SEL), smoke, bench, bench_quick, bench_pin (PIN_TILES), breakdown, prof,
# vtrace, pmc, sweep, ab (AB_SPECS), ablate, timeline, host, stamps_gemm (STAMP_SPEC)
STEPS=${STEPS:-tests bench prof}
run() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name (limit ${lim}s) $(date +%T)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc $(date +%T)"
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
for s in $STEPS; do
  case $s in
    tests)
      run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread
      rc=$?; [ $rc -le 1 ] || exit $rc ;;
    tests_sel)  # PYTEST_SEL: test files / node ids
      run pytest_sel 900 python -u -m pytest ${PYTEST_SEL} -m gpu -v -s -rf -p no:cacheprovider --timeout 300 --timeout-method thread
      rc=$?; [ $rc -le 1 ] || exit $rc ;;
    hostinfo)  # host facts the CPU baseline reads (num_cpus rule: affinity capped by the cgroup quota)
      { nproc; cat /sys/fs/cgroup/cpu.max 2>&1; cat /sys/fs/cgroup/cpu/cpu.cfs_quota_us 2>&1; echo "OMP=$OMP_NUM_THREADS"; } > gpurun_out/host.txt; cat gpurun_out/host.txt ;;
    sweep)
      run gemm_sweep 600 python tools/gemm_sweep.py || exit $? ;;
    ab)  # AB_SPECS: ';'-separated "M N K epi act tiles" (tools/gemm_ab.py, interleaved rounds in one process)
      IFS=';' read -ra SPECS <<< "${AB_SPECS}"
      for spec in "${SPECS[@]}"; do
        timeout -k 10 300 python3 tools/gemm_ab.py $spec ${AB_ROUNDS:-7} ${AB_ITERS:-20} >> gpurun_out/ab.log 2>&1 || exit $?
      done
      cat gpurun_out/ab.log ;;
    bench_pin)  # the vision leg with PIN_TILES pinned (q,o,f,p), BENCH_PIN_ARGS extra bench args
      run bench_pin_${PIN_TILES//,/_} 300 python bench.py --steps 20 --warmup 5 --tiles $PIN_TILES \
          --no-cpu-baseline --no-fp8 --no-text --no-e2e ${BENCH_PIN_ARGS:-} || exit $? ;;
    ablate)  # marginal step time of each trunk op (tools/ablate.py; needs lib/libclipgpu_ablate.so:
             # make variant VNAME=ablate VDEFS=-DCLIPGPU_ABLATE)
      CLIPGPU_LIB=$PWD/clip-embedder-rs_amd/lib/libclipgpu_ablate.so run ablate 600 python tools/ablate.py || exit $?
      cp gpurun_out/ablate.log gpurun_out/ablate.jsonl ;;
    bench_quick)  # the bench without the CPU leg
      run bench_quick 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $? ;;
    timeline)  # per-launch start / end of every trunk op with the lanes concurrent (tools/timeline.py)
      for spec in "vision 5 0" "vision 5 1" "text 3 0"; do
        run tl_$(echo $spec | tr ' ' _) 200 python tools/timeline.py $spec || exit $?
      done ;;
    host)  # host-side rates: copy pool, decoded-image entry point, u8 host path (tools/host_probe.py)
      run host_probe 300 python tools/host_probe.py || exit $? ;;
    stamps_gemm)  # K-step / epilogue cycles of one GEMM (needs lib/libclipgpu_stamps.so: make stamps;
                  # STAMP_SPEC "M N K epi act tile")
      CLIPGPU_LIB=$PWD/clip-embedder-rs_amd/lib/libclipgpu_stamps.so run stamps 300 python tools/gemm_stamps.py ${STAMP_SPEC:-} || exit $? ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
      run bench 600 python bench.py --steps 20 --warmup 5 || exit $? ;;
    breakdown)
      run breakdown 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp8 --no-text --no-e2e --breakdown || exit $? ;;
    vtrace)  # kernel trace of the vision leg alone; per-kernel stats of the timed steps only (tools/trace_timed.py)
      run vtrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/vtrace -o run --output-format csv -- \
          python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp8 --no-text --no-e2e --windows 0 || exit $?
      VLANES=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/vtrace.log') if l.startswith('{')][-1]['lanes_env'])") || exit 1
      python3 tools/trace_timed.py gpurun_out/vtrace/run_kernel_trace.csv 10 gpurun_out/vtrace_timed_kernels.txt $VLANES || exit $? ;;
    prof)
      run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
          python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit $?
      find gpurun_out/prof -name "*kernel_stats.csv" | head -3 ;;
    pmc)  # HBM bytes of the roofline kernel: FETCH_SIZE and WRITE_SIZE in separate passes,
          # GEMM tiles pinned to the ones the un-profiled bench autotuned (profiling skews tuning)
      TILES=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/bench.log') if l.startswith('{')][-1]['gemm_tiles_env'])") || exit 1
      LANES=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/bench.log') if l.startswith('{')][-1]['lanes_env'])") || exit 1
      for C in FETCH_SIZE WRITE_SIZE; do
        run pmc_$C 600 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_bench/$C -o run -- \
            python3 bench.py --steps 3 --warmup 1 --no-text --no-cpu-baseline --no-fp8 --no-e2e --windows 0 \
            --tiles $TILES --lanes $LANES || exit $?
      done
      cp profiles/pmc_c_fc.json gpurun_out/pmc_c_fc.json  # merged into (copy back to profiles/ after the call)
      for SITE in c_fc c_proj out_proj; do  # every site with a record; the bench reads its roofline kernel's
        ROWS=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/bench.log') if l.startswith('{')][-1]['gemm_sites']['$SITE']['rows_per_launch'])") || exit 1
        python3 tools/pmc_traffic.py gpurun_out/pmc_bench/FETCH_SIZE gpurun_out/pmc_bench/WRITE_SIZE \
            gpurun_out/pmc_c_fc.json $ROWS "${PMC_LABEL:-pmc run}: --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of bench.py --no-text, tiles $TILES" \
            "$TILES" $SITE || exit $?
      done ;;
  esac
done
echo "=== done"
