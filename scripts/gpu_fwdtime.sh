# Phase timing (s_memtime, block 0) of the c2 fused forward, x6 and fp32,
# then the c2 bench both ways
set -o pipefail
O=gpurun_out/fwdtime; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nnet.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for v in 1 0; do
KCNN_FWD_X6=$v KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_FWD_DEBUG=16 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/timing$v.log 2>&1 || exit 6
echo "x6=$v"; grep "fwd wave" $O/timing$v.log | tail -2
KCNN_FWD_X6=$v timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_x6$v.json > $O/bench_x6$v.log 2>&1 || exit 5
python -c "
import json;d=json.load(open('$O/bench_x6$v.json'));k=d.get('kernels') or {}
print('x6=$v', d['value'], d['ms_per_step'], {n:(v.get('ms'),v.get('mfma_frac')) for n,v in k.items() if 'conv' in n})"
done
