# SQ counter passes over a bench config (CFG, default c5) (one pass per counter group).
set -o pipefail
O=${1:-gpurun_out/pmc_c5}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MFMA" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/$tag -o run -- python bench.py --config ${CFG:-c5} --steps 1 --warmup 1 --no-cpu-baseline > $O/$tag.log 2>&1 || { echo "pmc $tag failed rc=$?" >> $O/fail.log; exit 3; }
done
echo done
