set -o pipefail
mkdir -p gpurun_out/pmc1
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc1/counters.txt 2>&1 || true
timeout -k 10 200 python scripts/microbench.py > gpurun_out/pmc1/micro.log 2>&1 || exit 3
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT TA_BUSY_avr TCP_TCC_WRITE_REQ_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc1/$tag -o run -- python scripts/microbench.py --reps 3 > gpurun_out/pmc1/$tag.log 2>&1 || echo "pmc $tag failed rc=$?" >> gpurun_out/pmc1/fail.log
done
echo done
