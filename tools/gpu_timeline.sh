set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for spec in "vision 5 0" "vision 5 1" "text 3 0"; do
  timeout -k 10 200 python tools/timeline.py $spec > gpurun_out/tl_$(echo $spec | tr ' ' _).log 2>&1 || { echo "fail $spec"; tail -5 gpurun_out/tl_*.log; exit 1; }
done
echo ok
