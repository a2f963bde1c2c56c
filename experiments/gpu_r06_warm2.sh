set -e
mkdir -p gpurun_out/r06warm2
for i in 1 2; do
  for w in 10 20 30 60 120; do
    timeout -k 10 240 python bench.py --warmup $w --steps 20 --no-cpu-baseline > gpurun_out/r06warm2/w${w}_$i.json
  done
done
timeout -k 10 240 python bench.py --config c5 --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/r06warm2/c5_w5.json
timeout -k 10 240 python bench.py --config c5 --warmup 30 --steps 20 --no-cpu-baseline > gpurun_out/r06warm2/c5_w30.json
timeout -k 10 240 python bench.py --config nnet --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/r06warm2/nnet_w5.json
timeout -k 10 240 python bench.py --config nnet --warmup 30 --steps 20 --no-cpu-baseline > gpurun_out/r06warm2/nnet_w30.json
