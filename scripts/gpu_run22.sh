set -o pipefail
O=gpurun_out/r22
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest.log; exit 3; }
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 > $O/c5.log 2>&1 || exit 4
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --config c5 --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 5
echo done
