# Phase timing of conv_bwd_x6q_kernel (experiment build) with parts of its
# work skipped (results wrong; timing only): 16 plain, +32 no image stores,
# +64 no MFMAs, +128 no splits, +256 no frame work
set -o pipefail
O=${1:-gpurun_out/x6qskip}; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
for d in 16 48 80 144 272 464; do
KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_BWD_X6P=2 KCNN_BWD_DEBUG=$d timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/t$d.log 2>&1 || exit 6
echo "== dbg $d"; grep "bwdx6q" $O/t$d.log | sort -k3,3n -k5,5n | awk '{print}' | head -40
done
