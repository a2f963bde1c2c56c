# x6 fused conv backward: component/nnet GPU tests, then the c2 bench with
# the x6 kernel and with the fp32 kernel (KCNN_BWD_X6=0), fused and unfused,
# c5, and a kernel profile of the default c2 step
set -o pipefail
O=${1:-gpurun_out/x6bwd}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_components.py tests/test_gpu_nnet.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -20; exit 3; }
for v in 1 0; do
  KCNN_BWD_X6=$v timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_x6$v.json > $O/bench_x6$v.log 2>&1 || exit 5
  KCNN_BWD_X6=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-fusion --json-out $O/bench_nf_x6$v.json > $O/bench_nf_x6$v.log 2>&1 || exit 5
  KCNN_BWD_X6=$v timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 --json-out $O/bench_c5_x6$v.json > $O/bench_c5_x6$v.log 2>&1 || exit 5
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
for f in bench_x61 bench_x60 bench_nf_x61 bench_nf_x60 bench_c5_x61 bench_c5_x60; do python -c "
import json;d=json.load(open('$O/$f.json'));k=d.get('kernels') or {}
print('$f', d['value'], d['ms_per_step'], {n:(v.get('ms'),v.get('mfma_frac')) for n,v in k.items() if 'conv' in n}, d.get('conv'), (d.get('scopes_ms_per_step') or {}).get('ConvolutionComponent::BackpropGradient'))"; done
head -8 $O/prof/run_kernel_stats.csv | cut -c1-120
