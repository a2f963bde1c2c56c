set -o pipefail
O=gpurun_out/r17
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_nnet.py -x -q -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest.log; exit 3; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 5
echo done
