# The f16x3 frame forward: determinism of repeated forwards, its range / Inf
# tests and the conv, fusion, GEMM and family suites, a kernel trace of the
# c2 step, the c2 bench with the f16x3 and the bf16x6 forward, and the
# forward's phase / store A/B in the timing build.
#   scripts/gpu_fwd_f16.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/fwdf16}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
REPS=30 bash experiments/diag_det2.sh > $O/det.log 2>&1 || { cat $O/det.log; exit 2; }
cat $O/det.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_fwd_f16.py tests/test_gpu_nnet.py tests/test_gpu_components.py tests/test_gpu_x6_range.py tests/test_gpu_families.py tests/test_gpu_gemm.py tests/test_gpu_threads.py "tests/test_gpu_fullsize.py::test_c2_bench_step" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest.log; tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c2.prof.log 2>&1 || exit 7
python scripts/kstats.py $(ls $O/c2/prof/*/run_kernel_stats.csv 2>/dev/null || ls $O/c2/prof/run_kernel_stats.csv) 25 16
for v in 2 1 2 1; do
  KCNN_FWD_X6=$v timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_$v.json > $O/bench_$v.log 2>&1 || exit 6
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('fwd_x6=$v', d['value'], d['ms_per_step'])"
done
if [ -n "$AB" ]; then DBGS="0 256 512" PHASE=16 bash scripts/gpu_fwd_ab.sh $O/ab || exit 8; fi
echo done
