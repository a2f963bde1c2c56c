set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for bk in 16 32; do
  KCNN_IGEMM2_BK=$bk timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --json-out gpurun_out/ab/bk$bk.json > gpurun_out/ab/bk$bk.log 2>&1 || exit 5
  python -c "import json;d=json.load(open('gpurun_out/ab/bk$bk.json'));print('bk$bk', d['value'], d['scopes_ms_per_step'])"
done
