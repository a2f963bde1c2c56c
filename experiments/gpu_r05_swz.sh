# r05: the implicit GEMM's conflict-free image swizzle -- its tests, the c5
# bench, the LDS counters and a trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05swz
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_igemm_f16.py tests/test_gpu_families.py tests/test_gpu_nnet.py tests/test_gpu_components.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 3; }
tail -1 $O/t.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5_$rep.json 2> $O/c5_$rep.err || exit 5
  python -c "import json;d=json.load(open('$O/c5_$rep.json'));print('c5', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --config nnet --steps 10 --warmup 3 --no-cpu-baseline > $O/nnet.json 2> $O/nnet.err || exit 5
python -c "import json;d=json.load(open('$O/nnet.json'));print('nnet', d['value'], d['ms_per_step'])"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc_lds -o run -- python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_lds.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || exit 7
echo done
