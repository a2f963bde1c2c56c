# A/B of one environment switch on the c5 bench: scripts/gpu_ab_env.sh VAR "v1 v2 ..."
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abenv
for v in $2; do
  env $1=$v timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --json-out gpurun_out/abenv/$v.json > gpurun_out/abenv/$v.log 2>&1 || exit 5
  python -c "import json;d=json.load(open('gpurun_out/abenv/$v.json'));print('$1=$v', d['value'], d['scopes_ms_per_step'])"
done
