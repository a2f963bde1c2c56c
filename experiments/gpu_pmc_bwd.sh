# SQ counters of the pooled conv backward (one rocprofv3 --pmc pass per set,
# each under its own time limit), for the kernel generations in VARS
# (KCNN_BWD_X6P on the experiment build)
set -o pipefail
O=${1:-gpurun_out/pmcbwd}; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $O/counters.txt | sort -u > $O/sq_counters.txt || true
S1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
S2="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES"
for v in ${VARS:-1 2}; do
  i=0
  for S in "$S1" "$S2"; do
    i=$((i+1))
    KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_BWD_X6P=$v timeout -s KILL 120 rocprofv3 --pmc $S --kernel-include-regex "conv_bwd" -d $O/v${v}_s$i -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/v${v}_s$i.log 2>&1 || { echo "pass v$v s$i failed"; tail -5 $O/v${v}_s$i.log; exit 7; }
  done
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for f in sorted(glob.glob(O + "/*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "conv_bwd" in r.get("Kernel_Name", ""):
            acc[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    print("==", f.split("/")[-3] if "/" in f else f)
    for (k, c), v in sorted(acc.items()):
        print("  %-40s %-26s %.4g (n=%d)" % (k, c, sum(v) / len(v), len(v)))
PY
