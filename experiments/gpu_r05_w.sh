# r05: full GPU suite, then the same-box c2 A/B against the pre-fixup library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r05w}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 3; }
tail -1 $O/pytest.txt
TAG=${TAG:-r05w}/ab bash experiments/gpu_r05_ab.sh
