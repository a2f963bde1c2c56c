# A/B of the fused forward's experiment switches (KCNN_FWD_DEBUG bits, the
# timing build): rocprof average of conv_fwd_regs_kernel per value, plus the
# per-phase s_memtime lines of block 0 (bit 16).
#   DBGS="0 256 512" scripts/gpu_fwd_ab.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/fwdab}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so
for d in ${DBGS:-0 256 512 768}; do
  KCNN_LIB=$LIB KCNN_FWD_DEBUG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$d -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/d$d.log 2>&1 || exit 7
  f=$(ls $O/d$d/*/run_kernel_stats.csv 2>/dev/null || ls $O/d$d/run_kernel_stats.csv)
  echo "dbg=$d $(python scripts/kstats.py $f 10 30 | grep conv_fwd_regs)"
done
if [ -n "$PHASE" ]; then
  KCNN_LIB=$LIB KCNN_FWD_DEBUG=$PHASE timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/phase.log 2>&1 || exit 6
  grep "fwd wave" $O/phase.log | tail -4
fi
