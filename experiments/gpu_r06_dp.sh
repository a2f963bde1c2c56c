# r06: the data-parallel step at world size 1 over RCCL (torchrun, one rank)
# beside the single-GPU step, at c4's per-rank shard (16384 frames) and c2's
# 4096, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-r06dp}; mkdir -p $O; export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
for B in 16384 4096; do for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --frames-per-gpu $B --json-out $O/single_${B}_$i.json > $O/single_${B}_$i.log 2>&1 || exit 5
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29511 bench.py --gpus 1 --no-cpu-baseline --frames-per-gpu $B --json-out $O/dp1_${B}_$i.json > $O/dp1_${B}_$i.log 2>&1 || exit 6
  python -c "
import json
a=json.load(open('$O/single_${B}_$i.json')); b=json.load(open('$O/dp1_${B}_$i.json'))
print('B $B single', a['value'], a['ms_per_step'], '| dp ws1', b['value'], b['ms_per_step'], 'overhead %.2f%%' % (100*(b['ms_per_step']/a['ms_per_step']-1)), b.get('dp'))"
done; done
