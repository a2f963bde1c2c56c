# r05 first GPU call: range tests (expected to fail before the guard), the RP
# and OOB fixes, the bench self-launch, the permlane / inline-asm determinism
# variants, the FC engines' error ratios and one c2 bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r05a
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest -p no:cacheprovider -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gemm.py tests/test_gpu_fwd_f16.py tests/test_gpu_nnet.py \
  "tests/test_gpu_dp.py::test_bench_gpus_n_launches_n_ranks" > gpurun_out/r05a/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; tail -40 gpurun_out/r05a/pytest.txt | grep -E "passed|failed|FAILED|ERROR" | tail -40
ok $rc || exit 3
for v in plv pla pln asm; do
  SHAPE=halfB REPS=60 KCNN_LIB=$PWD/kaldi-cnn_amd/libkcnn_$v.so timeout -k 10 150 python experiments/diag_det2.py \
    >> gpurun_out/r05a/det.txt 2>&1 || { echo "det $v rc $?"; exit 4; }
done
SHAPE=halfB REPS=60 timeout -k 10 150 python experiments/diag_det2.py >> gpurun_out/r05a/det.txt 2>&1 || exit 5
cat gpurun_out/r05a/det.txt
timeout -k 10 200 python scripts/gemm_error_ratio.py > gpurun_out/r05a/gemm_err.txt 2>&1 || exit 6
cat gpurun_out/r05a/gemm_err.txt
timeout -k 10 300 python bench.py --json-out gpurun_out/r05a/bench.json > gpurun_out/r05a/bench.log 2>&1 || exit 7
cat gpurun_out/r05a/bench.json
