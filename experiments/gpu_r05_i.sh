# r05: suspect-frame pool_count (list per block, no control words); tests,
# bench, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r05i}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool_stats.py tests/test_gpu_gemm.py tests/test_gpu_nnet.py tests/test_gpu_fwd_f16.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR|differs" $O/pytest.txt | head -20; tail -1 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || exit 5
python -c "
import json;d=json.load(open('$O/bench.json'));print('product', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 18
