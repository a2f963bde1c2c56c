set -o pipefail
O=gpurun_out/graph_a; rm -rf $O; mkdir -p $O
for a in "" "--no-graph" "" "--no-graph"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $a --json-out $O/b.json > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 3; }
  python -c "import json;d=json.load(open('$O/b.json'));print('$a', d['value'], d['ms_per_step'], d.get('hip_graph'), d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --json-out $O/c5.json > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 4; }
python -c "import json;d=json.load(open('$O/c5.json'));print('c5', d['value'], d['ms_per_step'], d.get('hip_graph'))"
timeout -k 10 300 python bench.py --config nnet --no-cpu-baseline --json-out $O/nnet.json > $O/nnet.log 2>&1 || { tail -20 $O/nnet.log; exit 4; }
python -c "import json;d=json.load(open('$O/nnet.json'));print('nnet', d['value'], d['ms_per_step'], d.get('hip_graph'))"
