# r05: pooled-output statistics without the column-min bytes (suspect-frame
# counting), reduce-kernel load restructure.  (1) the new exact-statistics
# test + suites; (2) reduce A/B (libkcnn_timing.so, KCNN_RED_DEBUG=1 drops
# the spread check); (3) bench + kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r05h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool_stats.py tests/test_gpu_gemm.py tests/test_gpu_nnet.py tests/test_gpu_fwd_f16.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR|differs" $O/pytest.txt | head -20; tail -1 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
for d in 0 1; do
  KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_RED_DEBUG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/red$d -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/red$d.log 2>&1 || exit 7
  echo "red dbg $d"; python scripts/kstats.py "$(find $O/red$d -name "*kernel_stats.csv" | head -1)" 40 18 | grep -E "reduce|pool_|stats" 
done
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || exit 5
python -c "
import json;d=json.load(open('$O/bench.json'));print('product', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 18
