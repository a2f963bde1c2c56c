# Same-box comparison of the pooled-backward generations: product library
# default, then the experiment build with KCNN_BWD_X6P = each of VARS
set -o pipefail
O=${1:-gpurun_out/bwdab}; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --no-cpu-baseline --json-out $O/prod.json > $O/prod.log 2>&1 || exit 5
python -c "import json;d=json.load(open('$O/prod.json'));print('product', d['value'], d['kernels']['conv_bwd_pooled']['ms'])"
for v in ${VARS:-1 2 1 2}; do
KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_BWD_X6P=$v KCNN_BWD_DEBUG=${DBG:-0} timeout -k 10 200 python bench.py --no-cpu-baseline --json-out $O/t$v.json > $O/t$v.log 2>&1 || exit 6
python -c "import json;d=json.load(open('$O/t$v.json'));print('x6p=$v', d['value'], d['kernels']['conv_bwd_pooled']['ms'])"
done
