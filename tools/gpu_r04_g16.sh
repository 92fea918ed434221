set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="bench pmc" bash tools/gpu_check.sh || exit $?
grep '^{' gpurun_out/bench.log | python3 -c "import sys,json; l=json.loads(sys.stdin.read()); print(json.dumps(l['roofline'])); print(json.dumps(l['gemm_sites']))"
echo ALLDONE
