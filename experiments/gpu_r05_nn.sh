# r05: bench lines after the parameter restore before the profiled pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r05nn
mkdir -p $O
for cfg in nnet c5 c2; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > $O/$cfg.json 2> $O/$cfg.err || exit 5
  python -c "import json;d=json.load(open('$O/$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d['profiled_ms_per_step'], d['roofline']['frac'], d.get('scopes_ms_per_step'))"
done
echo done
