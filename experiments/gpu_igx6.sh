# x6 long-kernel convs: GPU tests, then c5 / nnet benches
# with the x6 weight gradient on and off (KCNN_WGRAD_X6), and a c5 profile
set -o pipefail
O=${1:-gpurun_out/igx6}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 3; }
for v in 1 0; do
  for c in c5 nnet; do
    KCNN_WGRAD_X6=$v timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --json-out $O/b_${c}_$v.json > $O/b_${c}_$v.log 2>&1 || exit 5
    python -c "
import json;d=json.load(open('$O/b_${c}_$v.json'))
print('$c x6=$v', d['value'], d['ms_per_step'], d.get('conv'))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5prof -o run -- python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5prof.log 2>&1 || exit 6
head -12 $O/c5prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
