# A/B of two builds of libkcnn (LIBS, file names under kaldi-cnn_amd/): GPU
# tests on each, then c2 / c5 / nnet benches alternating the builds
set -o pipefail
O=${1:-gpurun_out/libab}
mkdir -p $O
export TMPDIR=/tmp
for lib in ${LIBS:-libkcnn.so}; do
  KCNN_LIB=$PWD/kaldi-cnn_amd/$lib timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_$lib.log 2>&1; rc=$?
  echo "$lib: $(tail -1 $O/pytest_$lib.log)"
  [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest_$lib.log | head -20; exit 3; }
done
for rep in 1 2; do
for lib in ${LIBS:-libkcnn.so}; do
  for c in ${CFGS:-c2 c5 nnet}; do
    KCNN_LIB=$PWD/kaldi-cnn_amd/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --json-out $O/b.json > $O/b.log 2>&1 || exit 5
    python -c "
import json;d=json.load(open('$O/b.json'));s=d.get('scopes_ms_per_step') or {};k=d.get('kernels') or {}
print('$c $lib', d['value'], d['ms_per_step'], {n:v.get('ms', v.get('ms_per_step')) for n,v in k.items()} if k else {a.split('::')[1]:b for a,b in s.items() if a.startswith('Conv')})"
  done
done
done
