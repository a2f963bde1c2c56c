# r05: the split-K fixup kernel (deferred recomputes): GEMM / component tests,
# then c2 and nnet.config bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05_fix
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_gpu_gemm.py tests/test_gpu_components.py -k "intra_group or c2_fc or fc_update or fast_path or ragged" \
  > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --json-out $O/c2.json > $O/c2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config nnet --no-cpu-baseline --json-out $O/nnet.json > $O/nnet.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --json-out $O/c5.json > $O/c5.log 2>&1 &&
echo done
