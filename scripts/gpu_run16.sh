set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "conv or Conv or golden or fd" > gpurun_out/pytest16.log 2>&1 || { echo "pytest_rc=$?" >> gpurun_out/pytest16.log; exit 3; }
: > gpurun_out/micro16.log
for v in "2 2" "3 2" "3 3" "3 4"; do
  set -- $v
  echo "variant=$1 bpc=$2" >> gpurun_out/micro16.log
  KCNN_FWD_VARIANT=$1 KCNN_FWD_BPC=$2 timeout -k 10 100 python scripts/microbench.py --reps 30 --only fwd >> gpurun_out/micro16.log 2>&1 || exit 5
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench16.log 2>&1 || exit 6
echo done
