# Fused Conv->Maxpool forward: parity tests, c2 / c5 bench, phase timing of block 0.
set -o pipefail
O=gpurun_out/fwdpool; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nnet.py tests/test_gpu_components.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for c in c2 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --json-out $O/b_$c.json > $O/b_$c.log 2>&1 || exit 5
  python -c "import json;d=json.load(open('$O/b_$c.json'));k=d.get('kernels',{});print('$c', d['value'], d['ms_per_step'], {n: k[n].get('ms') for n in k if 'ms' in k[n]}, d.get('scopes_ms_per_step',{}).get('ConvolutionComponent::PropagateMaxpool'))"
done
KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_FWD_DEBUG=16 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/timing.log 2>&1 || exit 6
grep "fwd wave" $O/timing.log | tail -4
