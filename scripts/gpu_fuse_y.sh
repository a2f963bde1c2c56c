# GPU suite, then the c2 / c5 benches with and without storing the fused conv output.
set -o pipefail
O=gpurun_out/fuse_y; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
for a in "" "--store-conv-out"; do
  for c in c2 c5; do
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline $a --json-out $O/b_${c}$a.json > $O/b_${c}$a.log 2>&1 || exit 5
    python -c "import json;d=json.load(open('$O/b_${c}$a.json'));k=d.get('kernels',{});print('$c $a', d['value'], d['ms_per_step'], {n: (k[n].get('ms'), k[n].get('GB/s')) for n in k if 'ms' in k[n]}, d.get('scopes_ms_per_step',{}).get('ConvolutionComponent::PropagateMaxpool'))"
  done
done
