set -o pipefail
O=gpurun_out/r23
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "conv or Conv or golden or fd" > $O/pytest.log 2>&1 || { echo "pytest_rc=$?" >> $O/pytest.log; exit 3; }
for d in 0; do
  KCNN_IGEMM2_DEBUG=$d timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$d -o run -- python bench.py --config c5 --steps 3 --warmup 1 > $O/prof$d.log 2>&1 || exit 5
done
echo done
