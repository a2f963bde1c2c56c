# igemm2 timing experiments (KCNN_IGEMM2_DEBUG: 1 = no operand loads, 2 = no LDS stores)
set -o pipefail
O=gpurun_out/ig2dbg
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
for d in 0 4 8 12; do
  KCNN_IGEMM2_DEBUG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$d -o run -- python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/d$d.log 2>&1 || exit 5
done
echo done
