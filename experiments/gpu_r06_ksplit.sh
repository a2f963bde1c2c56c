# r06: the f16x3 GEMM's split-K count forced (KCNN_F16X3_KSPLIT, experiments build
# libkcnn_ks.so of cu-gemm-f16x3.hip) against the chosen one, nnet.config and c2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r06ks; mkdir -p $O; export TMPDIR=/tmp
L=$PWD/kaldi-cnn_amd/libkcnn_ks.so
for i in 1 2; do for cfg in nnet c2; do for ks in 0 1 2; do
  KCNN_LIB=$L KCNN_F16X3_KSPLIT=$ks timeout -k 10 300 python bench.py --config $cfg --warmup 15 --steps 20 --no-cpu-baseline > $O/${cfg}_ks${ks}_$i.json 2> $O/${cfg}_ks${ks}_$i.err || exit 5
  python -c "import json;d=json.loads(open('$O/${cfg}_ks${ks}_$i.json').read().strip().splitlines()[-1]);print('$cfg ks$ks', d['value'], d['ms_per_step'])"
done; done; done
for ks in 0 1; do
  KCNN_LIB=$L KCNN_F16X3_KSPLIT=$ks timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nnet_ks$ks -o run -- python bench.py --config nnet --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_nnet_ks$ks.log 2>&1 || exit 6
  python scripts/kstats.py "$(find $O/prof_nnet_ks$ks -name "*kernel_stats.csv" | head -1)" 23 14
done
