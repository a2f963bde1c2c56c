# A/B of one environment switch on the c2 bench: scripts/gpu_ab_c2.sh VAR "v1 v2 ..."
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abc2
for v in $2; do
  env $1=$v timeout -k 10 300 python bench.py --no-cpu-baseline --json-out gpurun_out/abc2/$v.json > gpurun_out/abc2/$v.log 2>&1 || exit 5
  python -c "import json;d=json.load(open('gpurun_out/abc2/$v.json'));k=d['kernels'];print('$1=$v', d['value'], {n: k[n]['ms'] for n in k if 'ms' in k[n]})"
done
