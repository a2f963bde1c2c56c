# bf16x6 GEMM: correctness tests, then the c2 FC shapes (rocBLAS vs x6)
set -o pipefail
O=${1:-gpurun_out/gemm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1 || { tail -30 $O/pytest_gemm.log; exit 3; }
tail -1 $O/pytest_gemm.log
timeout -k 10 120 python scripts/gemm_bench.py > $O/gemm_bench.log 2>&1 || { cat $O/gemm_bench.log; exit 4; }
KCNN_X6_FAST=0 timeout -k 10 120 python scripts/gemm_bench.py > $O/gemm_bench_generic.log 2>&1 || exit 4
cat $O/gemm_bench.log; echo generic; cat $O/gemm_bench_generic.log
