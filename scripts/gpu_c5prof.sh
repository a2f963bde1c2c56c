# rocprofv3 kernel-trace stats of the c5 deep-stack bench.
set -o pipefail
O=${1:-gpurun_out/c5prof}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || exit 5
echo done
