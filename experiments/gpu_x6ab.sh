# A/B of a KCNN_* switch (VAR, values VALS) on the c5 / nnet benches after
# the component + nnet GPU tests; per-scope conv times
set -o pipefail
O=${1:-gpurun_out/x6ab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_components.py tests/test_gpu_nnet.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 3; }
for v in ${VALS:-1 0 1 0}; do
  for c in ${CFGS:-c5 nnet}; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --json-out $O/b.json > $O/b.log 2>&1 || exit 5
    python -c "
import json;d=json.load(open('$O/b.json'));s=d.get('scopes_ms_per_step') or {}
k=d.get('kernels') or {}
print('$c $VAR=$v', d['value'], d['ms_per_step'], {n:v.get('ms', v.get('ms_per_step')) for n,v in k.items()} if k else {k.split('::')[1]:v for k,v in s.items() if k.startswith('Conv')})" | tee -a $O/summary.txt
  done
done
