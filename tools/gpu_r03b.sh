set -eo pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "busy or bounce_modes or headline or tiles_match" > gpurun_out/r03b/pytest.log 2>&1 || { tail -30 gpurun_out/r03b/pytest.log; exit 1; }
tail -1 gpurun_out/r03b/pytest.log
timeout -k 10 120 rocprofv3 -L > gpurun_out/r03b/counters.txt 2>&1 || true
bash tools/profile.sh r03_c1 --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0
bash tools/profile.sh r03_c3 --config c3 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0
echo done
