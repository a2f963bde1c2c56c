# r05: (1) the pooled-vs-maxpool(Y) check of test_pooled_backward_across_frames
# repeated (it failed once in call e); (2) A/B of the register-pooled
# forward's new statistics (libkcnn_exp.so, KCNN_FWD_DEBUG bits: 1024 column
# min bytes, 2048 tap min, 4096 row min, 8192 checked sequence); (3) suites;
# (4) bench + kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r05g; mkdir -p $O; export TMPDIR=/tmp
for s in halfB_G96_2x1x4 win_2x1x4_G96 c5_P1_3x1x4; do for m in 1 2; do
  STACK=$s MODE=$m REPS=40 timeout -k 10 200 python experiments/diag_pool_vs_y.py >> $O/diag.txt 2>&1 || { echo "diag rc $?"; tail -5 $O/diag.txt; exit 4; }
done; done
grep -v amdgpu.ids $O/diag.txt | tail -20
for d in 0 1024 2048 4096 8192 15360 0; do
  KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_exp.so KCNN_FWD_DEBUG=$d timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/ab_$d.json > $O/ab_$d.log 2>&1 || exit 7
  python -c "
import json;d=json.load(open('$O/ab_$d.json'));k=d['kernels']
print('dbg $d', d['value'], d['ms_per_step'], k['conv_fwd_maxpool']['ms'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_nnet.py tests/test_gpu_fwd_f16.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR" $O/pytest.txt | head -20; tail -1 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || exit 5
python -c "
import json;d=json.load(open('$O/bench.json'));print('product', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 18
