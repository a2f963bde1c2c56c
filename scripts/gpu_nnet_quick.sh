# The GEMM, ReLU and network suites, then nnet.config's bench line and a
# kernel trace of its step (the FC GEMM / ReLU changes show there).
#   scripts/gpu_nnet_quick.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/nnetq}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_components.py tests/test_gpu_nnet2.py tests/test_gpu_nnet.py "tests/test_gpu_fullsize.py::test_c2_bench_step" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest.log; tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --config nnet --no-cpu-baseline --json-out $O/bench_nnet.json > $O/bench_nnet.log 2>&1 || exit 6
python -c "import json;d=json.load(open('$O/bench_nnet.json'));print('nnet', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nnet/prof -o run -- python bench.py --config nnet --steps 10 --warmup 3 --no-cpu-baseline > $O/nnet.prof.log 2>&1 || exit 7
python scripts/kstats.py $(ls $O/nnet/prof/*/run_kernel_stats.csv 2>/dev/null || ls $O/nnet/prof/run_kernel_stats.csv) 13 20
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_c2.json > $O/bench_c2.log 2>&1 || exit 8
python -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', d['value'], d['ms_per_step'])"
echo done
