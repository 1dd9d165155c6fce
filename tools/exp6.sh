set -e
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --config c4 --res 256 --spp 64 --steps 1 --warmup 1 > gpurun_out/c4_small.json 2> gpurun_out/c4.err
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c1_y.json 2>/dev/null
echo ok
