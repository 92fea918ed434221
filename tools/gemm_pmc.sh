# SQ / TA / TD counter passes over single GEMM launches (tools/gemm_ab.py, 1 round x 20 launches), one
# rocprofv3 --pmc run per pass and spec; medians per kernel via tools/pmc_summary.py.
# PMC_SPECS: ';'-separated "tag|M N K epi act tile".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_SALU SQ_LEVEL_WAVES SQ_INSTS_VALU TA_BUFFER_READ_LDS_WAVEFRONTS_sum TA_FLAT_READ_LDS_WAVEFRONTS_sum"
IFS=';' read -ra SPECS <<< "${PMC_SPECS}"
for sp in "${SPECS[@]}"; do
  tag=${sp%%|*}; spec=${sp#*|}
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_${tag}_$i -o run --output-format csv -- \
        python3 tools/gemm_ab.py $spec 1 20 > gpurun_out/pmc_${tag}_$i.log 2>&1 || { echo "pass $i of $tag failed"; tail -5 gpurun_out/pmc_${tag}_$i.log; exit 1; }
  done
  echo "== $tag: $spec"
  python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_ gemm_pipe
done
