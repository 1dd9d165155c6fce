set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c1_fused.json 2>/dev/null
LUMO_LDS_GRID=1024 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c1_fused_g1024.json 2>/dev/null
echo ok
