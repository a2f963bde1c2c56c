# The software-pipelined pooled backward: GPU suite, default bench, then A/B
# of the kernel generations on the experiment build (KCNN_BWD_X6P=0:
# conv_bwd_x6_kernel, 1: conv_bwd_x6p_kernel, 2: conv_bwd_x6q_kernel; VARS
# picks them) and the phase timing of each
set -o pipefail
O=${1:-gpurun_out/x6p}; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || exit 5
python -c "import json;d=json.load(open('$O/bench.json'));print('default', d['value'], {k:v['ms'] for k,v in d['kernels'].items() if 'ms' in v})"
VARS=${VARS:-1 2 1 2}
for v in $VARS; do
KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_BWD_X6P=$v timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_p$v.json > $O/bench_p$v.log 2>&1 || exit 5
python -c "import json;d=json.load(open('$O/bench_p$v.json'));print('x6p=$v', d['value'], {k:v['ms'] for k,v in d['kernels'].items() if 'ms' in v})"
done
for v in $(echo $VARS | tr " " "\n" | sort -u); do
KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_BWD_X6P=$v KCNN_BWD_DEBUG=16 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/timing$v.log 2>&1 || exit 6
grep "bwdx6" $O/timing$v.log | tail -40
done
