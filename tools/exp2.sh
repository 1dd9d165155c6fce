set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
for a in 2 3 5; do LUMO_BOUNCE_AHEAD=$a timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c1_ahead$a.json 2>/dev/null; done
for g in 1024 4096; do LUMO_LDS_GRID=$g timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c1_grid$g.json 2>/dev/null; done
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --res 512 --spp 256 > gpurun_out/s512.json 2>/dev/null
echo ok
