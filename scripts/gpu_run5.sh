set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_components.py -m gpu -x -q -p no:cacheprovider -k "backprop_gradient or conv_component" > gpurun_out/pytest_bwd.log 2>&1 || { echo "pytest_bwd_rc=$?" >> gpurun_out/pytest_bwd.log; exit 3; }
for d in 0 2 14; do
KCNN_BWD_DEBUG=$d timeout -k 10 120 python scripts/microbench.py --reps 20 --only bwd_fused > gpurun_out/micro5_$d.log 2>&1 || exit 4
done
echo done
