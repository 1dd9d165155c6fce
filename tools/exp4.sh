set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config c2 --spp 4 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c2_s4.json 2> gpurun_out/c2.err
timeout -k 10 400 python bench.py --config c3 --spp 4 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c3_s4.json 2> gpurun_out/c3.err
echo ok
