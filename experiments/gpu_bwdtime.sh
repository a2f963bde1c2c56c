# Phase timing (clock64, block 0, every wave) of the c2 fused backward
# (conv_bwd_x6_kernel; make timing build, KCNN_BWD_DEBUG=16)
set -o pipefail
O=${1:-gpurun_out/bwdtime}; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_BWD_DEBUG=16 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/timing.log 2>&1 || exit 6
grep "bwdx6 wave" $O/timing.log | tail -8
