# The f16x3 FC GEMM: its GPU tests (plus the re-entrancy, nnet2 and
# cross-frame pooled-backward tests), the fast kernel bitwise against the
# two-phase one (experiment build), the c2 FC shapes timed per engine, a
# kernel trace of the c2 step and the bench line.
#   scripts/gpu_f16x3.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/f16x3}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_x6_range.py tests/test_gpu_threads.py tests/test_gpu_nnet2.py "tests/test_gpu_nnet.py::test_pooled_backward_across_frames" "tests/test_gpu_fullsize.py::test_c2_bench_step" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest.log; tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
if [ -f kaldi-cnn_amd/libkcnn_timing.so ]; then
  VAR=KCNN_F16X3_FAST GEMM=2 timeout -k 10 300 python scripts/gemm_deep_bitwise.py > $O/fast_bitwise.log 2>&1 || { cat $O/fast_bitwise.log; exit 4; }
  cat $O/fast_bitwise.log
fi
GEMM_MODES=2,1 timeout -k 10 120 python scripts/gemm_bench.py > $O/gemm_bench.log 2>&1 || exit 4
cat $O/gemm_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c2.prof.log 2>&1 || exit 7
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || exit 6
python -c "import json;[print(f, json.load(open('$O/'+f))['value']) for f in ('bench.json',)]"
echo done
if [ -n "$CLOCK" ]; then
  CMD="python scripts/gemm_bench.py" GEMM_MODES=2 bash scripts/gpu_clock.sh $O/clock > $O/clock.txt 2>&1 || exit 8
  head -12 $O/clock.txt
fi
