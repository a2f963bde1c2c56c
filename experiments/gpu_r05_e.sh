# r05: same-box A/B of the r04 library (git aab7afe, built in a worktree)
# against the current one: c2 bench and kernel trace each, twice alternating;
# then the GEMM / nnet / fwd suites on the current library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r05e; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
for v in r04 cur; do
  L=$PWD/kaldi-cnn_amd/libkcnn.so; [ $v = r04 ] && L=$PWD/kaldi-cnn_amd/libkcnn_r04.so
  KCNN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_${v}_$rep.json > $O/bench_${v}_$rep.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', d['value'], d['ms_per_step'])"
done; done
for v in r04 cur; do
  L=$PWD/kaldi-cnn_amd/libkcnn.so; [ $v = r04 ] && L=$PWD/kaldi-cnn_amd/libkcnn_r04.so
  KCNN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_$v.log 2>&1 || exit 6
  echo "== $v"; python scripts/kstats.py "$(find $O/prof_$v -name "*kernel_stats.csv" | head -1)" 45 16
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_nnet.py tests/test_gpu_fwd_f16.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR" $O/pytest.txt | head -20; tail -1 $O/pytest.txt
