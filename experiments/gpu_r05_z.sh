# r05 (second session): f16x3 implicit GEMM with in-kernel fp32 recompute of
# rejected elements -- its tests, the tile census, c5 bench and trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05z4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_igemm_f16.py > $O/t_igemm.log 2>&1 || { tail -30 $O/t_igemm.log; exit 3; }
tail -2 $O/t_igemm.log
KCNN_LIB=kaldi-cnn_amd/libkcnn_timing.so KCNN_IGF16_DEBUG=1 timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_dbg.json 2> $O/c5_dbg.err || exit 5
grep "igemm f16x3" $O/c5_dbg.err | sort | uniq -c | sort -rn | head -20
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 6
cat $O/c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5_prof.log 2>&1 || exit 7
echo done
