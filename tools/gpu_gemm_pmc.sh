set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
T="timeout -k 10 300"
for K in 768 1536 3072 6144; do $T python tools/gemm_one.py 12800 3072 $K 0 1 3 20 || exit $?; done
for M in 2560 6400 12800 25600 51200; do $T python tools/gemm_one.py $M 3072 768 0 1 3 20 || exit $?; done
$T python tools/gemm_one.py 12800 3072 768 2 0 3 20 || exit $?
$T python tools/gemm_one.py 12800 3072 768 0 0 3 20 || exit $?
for P in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  n=$(echo $P | cut -d' ' -f1)
  $T rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc/$n -o run -- python3 tools/gemm_one.py 12800 3072 768 0 1 3 5 > gpurun_out/pmc/$n.log 2>&1 || exit $?
done
for P in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  n=sq_$(echo $P | cut -d' ' -f1)
  $T rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc/$n -o run -- python3 tools/gemm_one.py 4096 4096 4096 2 0 3 5 > gpurun_out/pmc/$n.log 2>&1 || exit $?
done
echo done
