# r05 final code: full GPU suite, smoke, c2 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 5
python -c "import json;d=json.load(open('$O/bench.json'));print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'])"
echo done
