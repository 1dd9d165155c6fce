set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bdpt.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_bdpt.log 2>&1
for v in 64 128; do timeout -k 10 600 python3 bench.py --config c4 --res 1024 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0 --max-vertices $v > gpurun_out/c4_v$v.json 2> gpurun_out/c4.err; done
echo ok
