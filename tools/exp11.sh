set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py --config c2 --spp 4 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c2_k.json 2> gpurun_out/c2.err
timeout -k 10 400 python bench.py --config c3 --spp 4 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c3_k.json 2> gpurun_out/c3.err
timeout -k 10 600 python3 bench.py --config c4 --res 1024 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c4_k.json 2> gpurun_out/c4.err
echo ok
