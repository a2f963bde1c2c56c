# SQ counters of the bf16x6 GEMM kernels at the c2 FC shapes (one pass per group)
set -o pipefail
O=${1:-gpurun_out/gemm_pmc}
mkdir -p $O
export TMPDIR=/tmp GEMM_MODES=1
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MFMA" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/$tag -o run -- python scripts/gemm_bench.py fwd > $O/$tag.log 2>&1 || { echo "pmc $tag failed rc=$?"; exit 3; }
done
python scripts/pmc_summary.py $O --match gemm_x6
