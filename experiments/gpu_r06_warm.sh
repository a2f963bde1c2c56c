set -e
mkdir -p gpurun_out/r06warm
for i in 1 2; do
  timeout -k 10 240 python bench.py --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/r06warm/w5_s20_$i.json
  timeout -k 10 240 python bench.py --warmup 30 --steps 20 --no-cpu-baseline > gpurun_out/r06warm/w30_s20_$i.json
  timeout -k 10 240 python bench.py --warmup 30 --steps 100 --no-cpu-baseline > gpurun_out/r06warm/w30_s100_$i.json
done
