# r05: c5 and nnet.config bench lines with the engine-relative rooflines, and
# the c2 line once more on the same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05_final
mkdir -p $O
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --json-out $O/c5.json > $O/c5.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config nnet --no-cpu-baseline --json-out $O/nnet.json > $O/nnet.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --json-out $O/c2.json > $O/c2.log 2>&1 &&
echo done
