# r06: tests, same-box A/B against the r05 library (c2), rocprof kernel
# stats and the FETCH / WRITE passes of the new library's c2 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r06b}; mkdir -p $O; export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR|Error|passed|failed" $O/pytest.txt | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
fi
for i in 1 2; do for lib in r05 new; do
  L=$PWD/kaldi-cnn_amd/libkcnn.so; [ $lib = r05 ] && L=$PWD/kaldi-cnn_amd/libkcnn_r05.so
  KCNN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline $BARGS --json-out $O/ab_${lib}_$i.json > $O/ab_${lib}_$i.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/ab_${lib}_$i.json'));print('$lib', d['value'], d['ms_per_step'], d['profiled_ms_per_step'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BARGS > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 20
if [ -n "$PMC" ]; then
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BARGS > $O/pmc_$c.log 2>&1 || exit 7
done
fi
echo done
