# r05: the f16x3 weight gradient (family 3) with 64 listed rejections per
# wave before a block falls back to bf16x6, against the wide bf16x6 default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05wg3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_igemm_f16.py -k wgrad > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 3; }
tail -1 $O/t.log
for rep in 1 2; do
for fam in 3 2; do
  KCNN_WGRAD_X6=$fam timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5_w${fam}_$rep.json 2> $O/c5_w${fam}_$rep.err || exit 5
  python -c "import json;d=json.load(open('$O/c5_w${fam}_$rep.json'));print('wgrad fam $fam', d['value'], d['ms_per_step'])"
done
done
KCNN_WGRAD_X6=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || exit 6
echo done
