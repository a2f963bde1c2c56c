# Round-1 validation + measurement on one MI355X (run via gpurun):
# tests, smoke, bench, kernel-trace profiles and PMC HBM traffic of the
# default (fused Conv->Maxpool) step and of the unfused step.
set -o pipefail
O=gpurun_out/r01b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1; echo "pytest_rc=$?" >> $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --no-cpu-baseline --no-fusion --json-out $O/bench_nofusion.json > $O/bench_nofusion.log 2>&1 || exit 4
for v in fused nofusion; do
  F=""; [ $v = nofusion ] && F="--no-fusion"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline $F > $O/$v.prof.log 2>&1 || exit 5
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/$v/pmc_$c -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline $F > $O/$v.pmc_$c.log 2>&1 || exit 6
  done
done
echo done
