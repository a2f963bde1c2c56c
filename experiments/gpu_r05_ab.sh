# r05: same-box A/B of the c2 step, the previous library (libkcnn_prev.so)
# against the current build, alternating; then the current build's kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r05ab}; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3; do for lib in prev new; do
  L=$PWD/kaldi-cnn_amd/libkcnn.so; [ $lib = prev ] && L=$PWD/kaldi-cnn_amd/libkcnn_prev.so
  KCNN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/ab_${lib}_$i.json > $O/ab_${lib}_$i.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/ab_${lib}_$i.json'));print('$lib', d['value'], d['ms_per_step'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
python scripts/kstats.py "$(find $O/prof -name "*kernel_stats.csv" | head -1)" 45 20
