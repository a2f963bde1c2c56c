# r05: same-box A/B of the implicit GEMM families on c5 (2 = f16x3 for the
# large convolutions, the default; 1 = bf16x6 everywhere), bench lines and
# kernel traces of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05ab2
mkdir -p $O
for rep in 1 2; do
for fam in 2 1; do
  KCNN_IGEMM_X6=$fam timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5_f${fam}_$rep.json 2> $O/c5_f${fam}_$rep.err || exit 5
  python -c "import json;d=json.load(open('$O/c5_f${fam}_$rep.json'));print('fam $fam', d['value'], d['ms_per_step'])"
done
done
for fam in 2 1; do
  KCNN_IGEMM_X6=$fam timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f$fam -o run -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_f$fam.log 2>&1 || exit 6
done
echo done
