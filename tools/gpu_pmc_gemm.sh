#!/bin/bash
# PMC passes over single GEMM configs (tools/gemm_one.py): one rocprofv3 --pmc run per counter
# group, each under its own time limit; output under gpurun_out/pmc_gemm/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_gemm
export TMPDIR=/tmp
CASES=${CASES:-"6400,3072,768,0,1,7 6400,768,3072,1,0,7"}
PMC_GROUPS=${PMC_GROUPS:-"SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_INST_LDS"}
if [ "${LIST:-0}" = 1 ]; then
  timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_gemm/counters.txt 2>&1 || exit 1
fi
i=0
for c in $CASES; do
  IFS=, read M N K EPI ACT TILE <<< "$c"
  g=0
  for grp in $PMC_GROUPS; do
    out=gpurun_out/pmc_gemm/c${i}_g${g}
    echo "=== case $c group $grp"
    timeout -s KILL 90 rocprofv3 --pmc ${grp//,/ } --output-format csv -d $out -o run -- \
        python3 tools/gemm_one.py $M $N $K $EPI $ACT $TILE 20 > $out.log 2>&1
    rc=$?
    tail -2 $out.log
    [ $rc -eq 0 ] || exit $rc
    g=$((g+1))
  done
  i=$((i+1))
done
echo "=== done"
