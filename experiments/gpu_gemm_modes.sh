# bf16x6 GEMM at the c2 FC shapes: plane kernel (pre-split operands), the
# default two-phase split kernel, and the one-block fast kernel
set -o pipefail
O=${1:-gpurun_out/gemm_modes}
mkdir -p $O
export TMPDIR=/tmp
GEMM_MODES=p,1,0 timeout -k 10 180 python scripts/gemm_bench.py > $O/modes.log 2>&1 || { cat $O/modes.log; exit 4; }
KCNN_X6_FAST=1 GEMM_MODES=1 timeout -k 10 120 python scripts/gemm_bench.py > $O/fast.log 2>&1 || { cat $O/fast.log; exit 4; }
cat $O/modes.log; echo fast; cat $O/fast.log
