set -o pipefail
O=${1:-gpurun_out/gemm_dbg}
mkdir -p $O
export GEMM_MODES=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1 || { tail -30 $O/pytest_gemm.log; exit 3; }
tail -1 $O/pytest_gemm.log
for d in ${DBGS:-0 3 0}; do
  echo "== dbg $d" >> $O/dbg.log
  KCNN_X6_DBG=$d timeout -k 10 120 python scripts/gemm_bench.py >> $O/dbg.log 2>&1 || exit 4
done
cat $O/dbg.log
