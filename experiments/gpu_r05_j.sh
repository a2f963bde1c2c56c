set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r05j; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python experiments/spread_census.py > $O/census.txt 2>&1 || { tail -5 $O/census.txt; exit 3; }
grep -v amdgpu $O/census.txt
