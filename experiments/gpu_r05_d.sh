# r05: suite + bench + kernel trace after the guard's cost cuts, and a census
# of the bench's spread groups.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r05d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python experiments/spread_census.py > $O/census.txt 2>&1 || exit 2
cat $O/census.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR" $O/pytest.txt | head -40; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || exit 5
python -c "
import json;d=json.load(open('$O/bench.json'));k=d['kernels']
print('product', d['value'], d['ms_per_step'], {n:v.get('ms', v.get('ms_per_step')) for n,v in k.items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 > $O/kstats.txt 2>&1; head -16 $O/kstats.txt
