# nnet.config bench + kernel profile
set -o pipefail
O=${1:-gpurun_out/nnetb}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config nnet --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 5; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --config nnet --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
echo done
