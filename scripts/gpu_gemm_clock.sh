# FC GEMM engines at the c2 shapes: timing (gemm_bench.py), then the effective
# clock and MFMA busy per kernel (GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES,
# SQ_BUSY_CYCLES in one --pmc pass with the kernel trace), then the c2 step.
#   scripts/gpu_gemm_clock.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/gemm_clock}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
GEMM_MODES=${MODES:-2,1} timeout -k 10 120 python scripts/gemm_bench.py > $O/gemm_bench.log 2>&1 || exit 4
cat $O/gemm_bench.log
CMD="python scripts/gemm_bench.py" GEMM_MODES=${MODES:-2,1} bash scripts/gpu_clock.sh $O/clock > $O/clock.txt 2>&1 || exit 5
cat $O/clock.txt | head -20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c2.prof.log 2>&1 || exit 7
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || exit 6
python -c "import json;print('bench', json.load(open('$O/bench.json'))['value'])"
