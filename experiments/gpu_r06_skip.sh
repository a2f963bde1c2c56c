# r06: the pooled backward's cost by part in the timing build (libkcnn_timing.so,
# KCNN_BWD_DEBUG skip bits: 32 no image stores, 64 no MFMAs, 128 no splits,
# 256 no frame work, 512 no gather, 1024 no col2im; wrong results, timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r06skip}; mkdir -p $O; export TMPDIR=/tmp
for d in ${DBGS:-0 64 128 512 1024 32 256 0}; do
  KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_timing.so KCNN_BWD_DEBUG=$d timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --json-out $O/skip_$d.json > $O/skip_$d.log 2>&1 || exit 5
  python -c "
import json;d=json.load(open('$O/skip_$d.json'));k=d['kernels'];print('dbg $d', 'bwd %.1f us' % (1e3*k['conv_bwd_pooled']['ms']), 'step', d['ms_per_step'])"
done
