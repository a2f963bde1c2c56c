# r05: counters of the c5 step (SQ groups, then HBM FETCH / WRITE passes):
# MFMA busy and traffic of the f16x3 implicit GEMM
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05pmc5
CFG=c5 bash scripts/gpu_pmc_cfg.sh $O || exit 3
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_$c.log 2>&1 || exit 4
done
python scripts/pmc_summary.py $O > $O/summary.txt 2>&1 || true
echo done
