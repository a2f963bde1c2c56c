# r06: run a list of test files (TESTS) on the GPU, -x, verbose log
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r06t}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 ${TLIM:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYARGS} > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR|Error|passed|failed" $O/pytest.txt | tail -12
exit $rc
