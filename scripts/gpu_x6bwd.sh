# x6 fused conv backward: component/nnet GPU tests, then the c2 bench with
# the x6 kernel and with the fp32 kernel (KCNN_BWD_X6=0), and a kernel profile
set -o pipefail
O=${1:-gpurun_out/x6bwd}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_components.py tests/test_gpu_nnet.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -20; exit 3; }
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_x6.json > $O/bench_x6.log 2>&1 || exit 5
KCNN_BWD_X6=0 timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_fp32.json > $O/bench_fp32.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python - <<'PY'
import json,csv,sys
O=sys.argv[1] if len(sys.argv)>1 else "gpurun_out/x6bwd"
PY
for f in bench_x6 bench_fp32; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['ms_per_step'], json.dumps(d['kernels']))"; done
head -8 $O/prof/run_kernel_stats.csv | cut -c1-150
