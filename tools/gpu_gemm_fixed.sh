set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
T="timeout -k 10 120"
for K in 256 768 1536 3072; do
  for E in "0 1" "0 0" "2 0" "1 0"; do $T python tools/gemm_one.py 12800 3072 $K $E 3 20 || exit $?; done
done
for M in 2048 4096 8192; do $T python tools/gemm_one.py $M 3072 768 0 1 3 20 || exit $?; done
echo done
