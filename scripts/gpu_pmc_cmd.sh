# SQ counter passes (one pass per counter group, each with the kernel trace)
# over any command: CMD (default: the c2 bench step, 3 steps).
#   CMD="python scripts/gemm_bench.py" scripts/gpu_pmc_cmd.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/pmc}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
CMD=${CMD:-python bench.py --steps 3 --warmup 1 --no-cpu-baseline}
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MFMA" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/$tag -o run -- $CMD > $O/$tag.log 2>&1 || { echo "pmc $tag failed rc=$?" >> $O/fail.log; exit 3; }
done
python scripts/pmc_summary.py $O > $O/summary.txt
echo done
