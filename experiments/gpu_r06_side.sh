# r06: the side stream -- its tests and the GPU tests around the nnet runtime,
# then same-box bench A/B with KCNN_SIDE_STREAM=0 / 1 (BARGS to bench.py),
# and (PROF=1) a kernel trace of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r06side}; mkdir -p $O; export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  ${TESTS:-tests/test_gpu_side_stream.py tests/test_gpu_nnet.py tests/test_gpu_threads.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py} > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
fi
for i in $(seq 1 ${ROUNDS:-2}); do for s in 0 1; do
  KCNN_SIDE_STREAM=$s timeout -k 10 300 python bench.py --no-cpu-baseline $BARGS --json-out $O/ab_${s}_$i.json > $O/ab_${s}_$i.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/ab_${s}_$i.json'));k=d.get('kernels',{});r=d.get('roofline',{})
print('side=$s', d['value'], d['ms_per_step'], d.get('profiled_ms_per_step'), r.get('achieved'), r.get('frac'))"
done; done
if [ -n "$PROF" ]; then for s in 0 1; do
  KCNN_SIDE_STREAM=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$s -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BARGS > $O/prof_$s.log 2>&1 || exit 6
  python scripts/kstats.py "$(find $O/prof_$s -name "*kernel_stats.csv" | head -1)" 45 ${TOPK:-8}
done; fi
echo done
