# r05: tests, then a same-box A/B of the round-4 library (libkcnn_r04.so,
# built from aab7afe) against this tree's, alternating, and a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r05l}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool_stats.py tests/test_gpu_components.py tests/test_gpu_gemm.py tests/test_gpu_nnet.py tests/test_gpu_fwd_f16.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR|differs" $O/pytest.txt | head -20; tail -1 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
for i in 1 2 3; do for lib in r04 new; do
  L=$PWD/kaldi-cnn_amd/libkcnn.so; [ $lib = r04 ] && L=$PWD/kaldi-cnn_amd/libkcnn_r04.so
  KCNN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/ab_${lib}_$i.json > $O/ab_${lib}_$i.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/ab_${lib}_$i.json'));print('$lib', d['value'], d['ms_per_step'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 18
