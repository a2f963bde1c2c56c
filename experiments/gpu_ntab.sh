# A/B of the streaming (nontemporal) accesses: the pool forward's loads and
# stores (KCNN_POOL_NT bit 1) and the fused conv + pool forward's Y stores
# (KCNN_CONV_Y_NT): GPU kernel / component / stack tests, then the
# --no-fusion and --store-conv-out c2 benches with the defaults and with both off
set -o pipefail
O=${1:-gpurun_out/ntab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_components.py tests/test_gpu_nnet.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for rep in 1 2; do for v in "2 1" "0 0"; do set -- $v
  for mode in --no-fusion --store-conv-out; do
    KCNN_POOL_NT=$1 KCNN_CONV_Y_NT=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $mode --json-out $O/b.json > $O/b.log 2>&1 || exit 5
    python -c "
import json;d=json.load(open('$O/b.json'));k=d['kernels']
print('pool_nt=$1 y_nt=$2 $mode', d['value'], {n:(v.get('ms'),v.get('hbm_frac')) for n,v in k.items() if n!='fc_gemms'})" | tee -a $O/summary.txt
  done
done; done
