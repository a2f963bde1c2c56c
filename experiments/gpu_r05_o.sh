# r05: the f16x3 GEMM's per-tile overhead at c2's data-gradient shape
# (experiments/gemm_k_sweep.py) in the experiment build, KCNN_GEMM_DEBUG:
# 1 no C stores, 2 nontemporal C stores, 4 no statistics loads (timing only),
# 8 C through LDS with 16-B stores
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r05o; mkdir -p $O; export TMPDIR=/tmp
TL=$PWD/kaldi-cnn_amd/libkcnn_timing.so
for d in 0 8 1 2 4 5; do
  KCNN_LIB=$TL KCNN_GEMM_DEBUG=$d timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ks$d -o run -- python experiments/gemm_k_sweep.py > $O/ks$d.log 2>&1 || exit 8
  python - <<PY
import csv, glob, statistics
f = glob.glob("$O/ks$d/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "fast_kernel" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print("dbg $d", [("K%d" % k, round(statistics.median(d[20 * i + 3:20 * (i + 1)]), 1)) for i, k in enumerate((256, 512, 1024, 2048))])
PY
done
