# r05 (second session): flagged-tile census of the f16x3 implicit GEMM on c5
# (experiment build, KCNN_IGF16_DEBUG=1), then the c5 bench with the product
# library and its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05y
mkdir -p $O
KCNN_LIB=kaldi-cnn_amd/libkcnn_timing.so KCNN_IGF16_DEBUG=1 timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5_dbg.json 2> $O/c5_dbg.err || exit 5
grep "igemm f16x3" $O/c5_dbg.err | sort | uniq -c | sort -rn | head -20
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 6
cat $O/c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5_prof.log 2>&1 || exit 7
echo done
