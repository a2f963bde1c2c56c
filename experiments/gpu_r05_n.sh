# r05: tests; same-box A/B against r04; kernel trace; the product GEMM's
# per-tile overhead (experiments/gemm_k_sweep.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r05n}; mkdir -p $O; export TMPDIR=/tmp
if [ -z "$SKIPTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool_stats.py tests/test_gpu_components.py tests/test_gpu_gemm.py tests/test_gpu_nnet.py tests/test_gpu_fwd_f16.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR|differs" $O/pytest.txt | head -20; tail -1 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
fi
for i in 1 2; do for lib in r04 new; do
  L=$PWD/kaldi-cnn_amd/libkcnn.so; [ $lib = r04 ] && L=$PWD/kaldi-cnn_amd/libkcnn_r04.so
  KCNN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/ab_${lib}_$i.json > $O/ab_${lib}_$i.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/ab_${lib}_$i.json'));print('$lib', d['value'], d['ms_per_step'])"
done; done
if [ -n "$NNET" ]; then
  timeout -k 10 300 python bench.py --config nnet --no-cpu-baseline --json-out $O/nnet.json > $O/nnet.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/nnet.json'));print('nnet', d['value'], d['ms_per_step'])"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 20
if [ -n "$KSWEEP" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ksweep -o run -- python experiments/gemm_k_sweep.py > $O/ksweep.log 2>&1 || exit 8
python - <<PY
import csv, glob, statistics
f = glob.glob("$O/ksweep/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "fast_kernel" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
for i, k in enumerate((256, 512, 1024, 2048)):
    x = d[20 * i + 3:20 * (i + 1)]
    print("K", k, "fast kernel median us", round(statistics.median(x), 1))
PY
fi
