# Full GPU validation of the tree: tests, smoke, bench c2 and c5.
#   scripts/gpu_check.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/check}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest_gpu.log; exit 3; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || exit 5
timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline --json-out $O/bench_c5.json > $O/bench_c5.log 2>&1 || exit 6
echo done
