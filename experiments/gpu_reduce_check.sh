set -o pipefail
O=gpurun_out/redq; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_components.py "tests/test_gpu_fullsize.py::test_c2_bench_step" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 7
python scripts/kstats.py $(ls $O/prof/*/run_kernel_stats.csv 2>/dev/null || ls $O/prof/run_kernel_stats.csv) 25 8
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/b$i.json > $O/b$i.log 2>&1 || exit 6; python -c "import json;d=json.load(open('$O/b$i.json'));print('c2', d['value'], d['ms_per_step'])"; done
