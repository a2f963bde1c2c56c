# A/B of pooled-backward builds (LIBS under kaldi-cnn_amd/): the fusion
# and pooled-backward GPU tests on each, then c2 benches alternating the
# builds, reporting the pooled backward's launch time and the step.
#   LIBS="libkcnn.so libkcnn_ga2.so" scripts/gpu_bwd_var.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/bwdvar}
mkdir -p $O
export TMPDIR=/tmp
for lib in ${LIBS:-libkcnn.so}; do
  KCNN_LIB=$PWD/kaldi-cnn_amd/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_nnet.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_$lib.log 2>&1 || { echo "$lib: tests failed"; tail -30 $O/pytest_$lib.log; exit 3; }
  echo "$lib: $(tail -1 $O/pytest_$lib.log)"
done
for rep in 1 2 3; do
for lib in ${LIBS:-libkcnn.so}; do
  KCNN_LIB=$PWD/kaldi-cnn_amd/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 10 --json-out $O/b.json > $O/b.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/b.json'));k=d['kernels']
print('$lib', d['value'], d['ms_per_step'], 'bwd', k['conv_bwd_pooled']['ms'], 'fwd', k['conv_fwd_maxpool']['ms'])"
done
done
