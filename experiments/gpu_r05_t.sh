# r05: full GPU suite, then c2 / nnet.config / c5 bench lines and the
# nnet.config kernel trace (all-zero groups unchecked, the split-K fixup)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r05t}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 3; }
tail -1 $O/pytest.txt
for c in c2 nnet c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --json-out $O/$c.json > $O/$c.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/$c.json'));print('$c', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nprof -o run -- python bench.py --config nnet --steps 10 --warmup 3 --no-cpu-baseline > $O/nprof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/nprof -name "*kernel_stats.csv" | head -1)" 16 13
