set -o pipefail
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MFMA" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc2/$tag -o run -- python scripts/microbench.py --reps 3 --only fwd,bwd_fused > gpurun_out/pmc2/$tag.log 2>&1 || { echo "pmc $tag failed rc=$?" >> gpurun_out/pmc2/fail.log; exit 3; }
done
echo done
