# r05: nnet.config's FC GEMM operand census over training steps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r05q; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u experiments/spread_census_nnet.py > $O/census.txt 2>&1; rc=$?
grep -v amdgpu $O/census.txt | tail -60; exit $rc
