# r05: experiment -- the f16x3 implicit GEMM splitting the next step between
# its two MFMA halves in every wave (KCNN_IGF16_EARLY=1, timing build) vs the
# default order; c5 bench lines alternating, then a trace of each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05early
mkdir -p $O
export KCNN_LIB=kaldi-cnn_amd/libkcnn_timing.so
for rep in 1 2; do
for e in 1 0; do
  KCNN_IGF16_EARLY=$e timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5_e${e}_$rep.json 2> $O/c5_e${e}_$rep.err || exit 5
  python -c "import json;d=json.load(open('$O/c5_e${e}_$rep.json'));print('early $e', d['value'], d['ms_per_step'])"
done
done
for e in 1 0; do
  KCNN_IGF16_EARLY=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e$e -o run -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_e$e.log 2>&1 || exit 6
done
echo done
