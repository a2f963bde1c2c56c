# r05: GEMM / component tests with the fixup's early exit, then the same-box
# A/B of c2 against the pre-fixup library (experiments/gpu_r05_ab.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r05u}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_gpu_gemm.py tests/test_gpu_components.py tests/test_gpu_nnet.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
TAG=${TAG:-r05u}/ab bash experiments/gpu_r05_ab.sh
