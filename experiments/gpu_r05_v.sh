# r05: fixup grid 128: storm timing (experiments/fixup_storm.py), GEMM tests,
# c2 A/B against the pre-fixup library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r05v}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u experiments/fixup_storm.py > $O/storm.log 2>&1 || { tail -20 $O/storm.log; exit 4; }
cat $O/storm.log | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_gpu_gemm.py tests/test_gpu_components.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
TAG=${TAG:-r05v}/ab bash experiments/gpu_r05_ab.sh
