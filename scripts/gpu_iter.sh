# Iteration run: a filtered GPU test subset, then a bench line.
#   scripts/gpu_iter.sh <outdir> "<pytest -k expr>" "<bench args>"
set -o pipefail
O=${1:-gpurun_out/iter}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$2" > $O/pytest.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest.log; tail -30 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline $3 --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 5; }
cat $O/bench.json
