# r05: f16x3 weight gradient as family 3 (not default): its tests, the
# families / range tests, c5 default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05wg2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_igemm_f16.py tests/test_gpu_families.py tests/test_gpu_x6_range.py tests/test_abi.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 3; }
tail -1 $O/t.log
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 5
python -c "import json;d=json.load(open('$O/c5.json'));print('c5', d['value'], d['ms_per_step'])"
echo done
