set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c1_buck.json 2>/dev/null
LUMO_BUCKETS=0 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c1_nobuck.json 2>/dev/null
timeout -k 10 400 python bench.py --config c3 --spp 4 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c3_buck.json 2>/dev/null
LUMO_BUCKETS=0 timeout -k 10 400 python bench.py --config c3 --spp 4 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c3_nobuck.json 2>/dev/null
echo ok
