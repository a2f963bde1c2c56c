# The GPU suite N times in one call (intermittent numerical mismatches, not
# faults: a failing run prints its first failures and the loop goes on only
# while runs pass)
set -o pipefail
O=${1:-gpurun_out/rep}
mkdir -p $O
export TMPDIR=/tmp
for i in $(seq 1 ${N:-3}); do
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_$i.log 2>&1; rc=$?
  echo "run $i: $(tail -1 $O/pytest_$i.log)"
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_$i.log | head -10; exit 3; }
done
exit 0
