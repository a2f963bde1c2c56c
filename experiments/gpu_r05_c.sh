# r05 third call: the whole GPU suite with counted spread groups, the c2
# bench and its kernel trace, and an A/B of the register-pooled forward's
# new statistics (experiment build: KCNN_FWD_DEBUG 1024 drops the column min
# bytes, 2048 the position columns' min).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r05c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR" $O/pytest.txt | head -40; tail -2 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || exit 5
python -c "
import json;d=json.load(open('$O/bench.json'));k=d['kernels']
print('product', d['value'], d['ms_per_step'], {n:v.get('ms', v.get('ms_per_step')) for n,v in k.items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 > $O/kstats.txt 2>&1; head -16 $O/kstats.txt
for d in 0 1024 2048 3072 0; do
  KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_FWD_DEBUG=$d timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/ab_$d.json > $O/ab_$d.log 2>&1 || exit 7
  python -c "
import json;d=json.load(open('$O/ab_$d.json'));k=d['kernels']
print('dbg $d', d['value'], d['ms_per_step'], k['conv_fwd_maxpool']['ms'])"
done
