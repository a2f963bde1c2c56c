# The f16x3 FC GEMM: its GPU tests, the c2 FC shapes timed per engine, a
# kernel trace of the default engine, and the c2 bench step.
#   scripts/gpu_f16x3.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/f16x3}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_x6_range.py tests/test_gpu_threads.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest.log; tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
GEMM_MODES=1,2,0 timeout -k 10 120 python scripts/gemm_bench.py > $O/gemm_bench.log 2>&1 || exit 4
cat $O/gemm_bench.log
GEMM_MODES=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gprof -o run -- python scripts/gemm_bench.py > $O/gprof.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || exit 6
KCNN_GEMM=1 timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_x6.json > $O/bench_x6.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c2.prof.log 2>&1 || exit 7
python -c "import json;[print(f, json.load(open('$O/'+f))['value']) for f in ('bench.json','bench_x6.json')]"
echo done
