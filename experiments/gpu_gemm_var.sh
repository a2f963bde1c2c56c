# bf16x6 GEMM build variants (KCNN_LIB): tests + c2 FC shape times
set -o pipefail
O=${1:-gpurun_out/gemm_var}
mkdir -p $O
export GEMM_MODES=1
for v in ${VARS:-libkcnn.so}; do
  echo "== $v" >> $O/var.log
  KCNN_LIB=$PWD/kaldi-cnn_amd/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1; echo "pytest rc=$? $(tail -1 $O/pytest_$v.log)" >> $O/var.log
  KCNN_LIB=$PWD/kaldi-cnn_amd/$v timeout -k 10 120 python scripts/gemm_bench.py >> $O/var.log 2>&1 || exit 4
done
cat $O/var.log
