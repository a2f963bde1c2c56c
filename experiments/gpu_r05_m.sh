# r05: tests; the job-loop GEMM kernel variant (libkcnn_jl.so, an experiment build of
# KCNN_F16X3_PERSIST=1) under the GEMM tests; same-box A/B against r04;
# kernel traces of the product and of the persistent grid; the GEMM's
# per-tile overhead (experiments/gemm_k_sweep.py) for both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r05m; mkdir -p $O; export TMPDIR=/tmp
TL=$PWD/kaldi-cnn_amd/libkcnn_jl.so
if [ -z "$SKIPTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool_stats.py tests/test_gpu_components.py tests/test_gpu_gemm.py tests/test_gpu_nnet.py tests/test_gpu_fwd_f16.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR|differs" $O/pytest.txt | head -20; tail -1 $O/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
KCNN_LIB=$TL KCNN_F16X3_PERSIST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_components.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_persist.txt 2>&1
rc=$?; echo "persist pytest rc $rc"; grep -E "FAILED|ERROR" $O/pytest_persist.txt | head; tail -1 $O/pytest_persist.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
fi
for i in 1 2; do for lib in r04 new; do
  L=$PWD/kaldi-cnn_amd/libkcnn.so; [ $lib = r04 ] && L=$PWD/kaldi-cnn_amd/libkcnn_r04.so
  KCNN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/ab_${lib}_$i.json > $O/ab_${lib}_$i.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/ab_${lib}_$i.json'));print('$lib', d['value'], d['ms_per_step'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 20
for pe in 0 1; do
  KCNN_LIB=$TL KCNN_F16X3_PERSIST=$pe timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p$pe -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_p$pe.log 2>&1 || exit 6
  echo "timing lib persist $pe"; python scripts/kstats.py "$(find $O/prof_p$pe -name "*kernel_stats.csv" | head -1)" 45 4
  KCNN_LIB=$TL KCNN_F16X3_PERSIST=$pe timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ksweep$pe -o run -- python experiments/gemm_k_sweep.py > $O/ksweep$pe.log 2>&1 || exit 8
  python - <<PY
import csv, glob, statistics
f = glob.glob("$O/ksweep$pe/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "fast_kernel" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
for i, k in enumerate((256, 512, 1024, 2048)):
    x = d[20 * i + 3:20 * (i + 1)]
    print("persist $pe K", k, "fast kernel median us", round(statistics.median(x), 1))
PY
done
