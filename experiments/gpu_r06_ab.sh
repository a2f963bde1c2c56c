# r06: same-box A/B of library builds (LIBS: names of kaldi-cnn_amd/libkcnn_<name>.so,
# "new" = libkcnn.so), ROUNDS alternations, BARGS passed to bench.py; then
# optionally (PROF=1) the rocprof kernel stats of the new library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r06ab}; mkdir -p $O; export TMPDIR=/tmp
for i in $(seq 1 ${ROUNDS:-2}); do for lib in ${LIBS:-new}; do
  L=$PWD/kaldi-cnn_amd/libkcnn_$lib.so; [ $lib = new ] && L=$PWD/kaldi-cnn_amd/libkcnn.so
  KCNN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline $BARGS --json-out $O/ab_${lib}_$i.json > $O/ab_${lib}_$i.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/ab_${lib}_$i.json'));k=d.get('kernels',{});print('$lib', d['value'], d['ms_per_step'], d['profiled_ms_per_step'], k.get('fc_gemms',{}).get('ms_per_step'))"
done; done
if [ -n "$PROF" ]; then
# PROF=all: every library of LIBS in turn (KCNN_LIB), else the new one
PL=new; [ "$PROF" = all ] && PL="$LIBS"
for lib in $PL; do
  L=$PWD/kaldi-cnn_amd/libkcnn_$lib.so; [ $lib = new ] && L=$PWD/kaldi-cnn_amd/libkcnn.so
  echo "== $lib"
  KCNN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lib -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BARGS > $O/prof_$lib.log 2>&1 || exit 6
  python scripts/kstats.py "$(find $O/prof_$lib -name "*kernel_stats.csv" | head -1)" 45 ${TOPK:-8}
done
fi
echo done
