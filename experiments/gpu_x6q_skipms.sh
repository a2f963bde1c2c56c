# conv_bwd_x6q_kernel time (bench.py's HIP-event scope, experiment build) with
# parts of its work skipped (results wrong; timing only): 32 no image stores,
# 64 no MFMAs, 128 no splits, 256 no frame work (gather, col2im, map, Z)
set -o pipefail
O=${1:-gpurun_out/x6qms}; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
for d in ${DS:-0 32 64 128 256 96 160 288 384 224 480}; do
KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_BWD_X6P=${V:-2} KCNN_BWD_DEBUG=$d timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --json-out $O/b$d.json > $O/b$d.log 2>&1 || exit 6
python -c "import json;d=json.load(open('$O/b$d.json'));print('skip $d', d['kernels']['conv_bwd_pooled']['ms'])"
done
