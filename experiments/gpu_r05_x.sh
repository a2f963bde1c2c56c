# r05 (second session): the f16x3 implicit GEMM (igemm_x6 family 2) --
# its tests, the families / range / c5 stack tests, then the c5 bench with a
# kernel trace and the c2 / nnet.config bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_igemm_f16.py > $O/t_igemm.log 2>&1 || { tail -30 $O/t_igemm.log; exit 3; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_families.py tests/test_gpu_x6_range.py tests/test_gpu_components.py \
  tests/test_gpu_nnet.py > $O/t_more.log 2>&1 || { tail -30 $O/t_more.log; exit 4; }
tail -3 $O/t_more.log
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 5
cat $O/c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5_prof.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --config nnet --steps 10 --warmup 3 --no-cpu-baseline > $O/nnet.json 2> $O/nnet.err || exit 7
cat $O/nnet.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 8
cat $O/c2.json
echo done
