set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 600 python3 bench.py --config c4 --res 1024 --spp 8 --steps 1 --warmup 1 > gpurun_out/c4_n.json 2> gpurun_out/c4.err
echo ok
