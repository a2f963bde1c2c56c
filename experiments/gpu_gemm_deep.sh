# The two-deep-prefetch FC GEMM (gemm_x6d_kernel): GPU suite, then the c2
# bench A/B against gemm_x6_kernel on the experiment build (KCNN_X6_DEEP=0/1)
set -o pipefail
O=${1:-gpurun_out/x6d}; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python bench.py --no-cpu-baseline --json-out $O/prod.json > $O/prod.log 2>&1 || exit 5
python -c "import json;d=json.load(open('$O/prod.json'));print('product', d['value'], d['ms_per_step'], d['kernels']['fc_gemms']['ms_per_step'])"
for v in ${VARS:-0 1 0 1}; do
KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_X6_DEEP=$v timeout -k 10 200 python bench.py --no-cpu-baseline --json-out $O/t$v.json > $O/t$v.log 2>&1 || exit 6
python -c "import json;d=json.load(open('$O/t$v.json'));print('deep=$v', d['value'], d['ms_per_step'], d['kernels']['fc_gemms']['ms_per_step'])"
done
