# Larger per-GPU batches: c4's 16384 frames/GPU for every config, and c2 at 131072.
set -o pipefail
O=gpurun_out/sizes
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
for cfg in c2 c5 nnet; do
  timeout -k 10 300 python bench.py --config $cfg --frames-per-gpu 16384 --steps 5 --warmup 2 --no-cpu-baseline --json-out $O/$cfg.json > $O/$cfg.log 2>&1 || { tail -5 $O/$cfg.log; exit 5; }
  python -c "import json; d=json.load(open('$O/$cfg.json')); print('$cfg', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --frames-per-gpu 131072 --steps 3 --warmup 1 --no-cpu-baseline --json-out $O/c2big.json > $O/c2big.log 2>&1 || { tail -5 $O/c2big.log; exit 6; }
python -c "import json; d=json.load(open('$O/c2big.json')); print('c2 131072', d['value'], d['ms_per_step'], d['roofline']['frac'])"
