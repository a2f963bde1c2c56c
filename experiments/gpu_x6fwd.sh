# x6 conv forward: component/nnet/golden GPU tests, then the c2 bench with
# the x6 forward and with the fp32 kernel (KCNN_FWD_X6=0), fused and unfused, c5
set -o pipefail
O=${1:-gpurun_out/x6fwd}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_components.py tests/test_gpu_nnet.py tests/test_gpu_golden.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 3; }
for v in 1 0; do
  KCNN_FWD_X6=$v timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_x6$v.json > $O/bench_x6$v.log 2>&1 || exit 5
  KCNN_FWD_X6=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-fusion --json-out $O/bench_nf_x6$v.json > $O/bench_nf_x6$v.log 2>&1 || exit 5
  KCNN_FWD_X6=$v timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 --json-out $O/bench_c5_x6$v.json > $O/bench_c5_x6$v.log 2>&1 || exit 5
done
for f in bench_x61 bench_x60 bench_nf_x61 bench_nf_x60 bench_c5_x61 bench_c5_x60; do python -c "
import json;d=json.load(open('$O/$f.json'));k=d.get('kernels') or {}
print('$f', d['value'], d['ms_per_step'], {n:(v.get('ms'),v.get('mfma_frac')) for n,v in k.items() if 'conv' in n}, (d.get('scopes_ms_per_step') or {}).get('ConvolutionComponent::PropagateMaxpool'))"; done
