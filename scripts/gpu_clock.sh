# Effective clock per kernel of the c2 step: GRBM_GUI_ACTIVE / 8 XCDs over
# the dispatch duration (kernel trace in the same pass), plus MFMA busy
set -o pipefail
O=${1:-gpurun_out/clock}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/p -o run -- ${CMD:-python bench.py --steps 3 --warmup 2 --no-cpu-baseline ${ARGS}} > $O/p.log 2>&1 || exit 3
python scripts/clock_summary.py $O
