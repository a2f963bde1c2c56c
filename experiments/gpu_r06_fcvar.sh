# r06: the FC GEMM shapes (experiments/fc_shapes.py) with each library of
# LIBS ("new" = libkcnn.so), event timing and the per-kernel trace stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r06fcvar}; mkdir -p $O; export TMPDIR=/tmp
for lib in ${LIBS:-new}; do
  L=$PWD/kaldi-cnn_amd/libkcnn_$lib.so; [ $lib = new ] && L=$PWD/kaldi-cnn_amd/libkcnn.so
  echo "== $lib"
  KCNN_LIB=$L timeout -k 10 120 python experiments/fc_shapes.py 20 || exit 5
  KCNN_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lib -o run -- python experiments/fc_shapes.py 20 > $O/prof_$lib.log 2>&1 || exit 6
  python scripts/kstats.py "$(find $O/prof_$lib -name "*kernel_stats.csv" | head -1)" 1 ${TOPK:-6}
done
echo done
