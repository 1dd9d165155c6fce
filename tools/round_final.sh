set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
bash tools/profile.sh r01d --steps 1 --warmup 0 --cpu-baseline 0
timeout -k 10 500 python3 bench.py --config c2 --spp 4 --steps 1 --warmup 1 > gpurun_out/c2_final.json 2> gpurun_out/c2.err
timeout -k 10 500 python3 bench.py --config c3 --spp 4 --steps 1 --warmup 1 > gpurun_out/c3_final.json 2> gpurun_out/c3.err
timeout -k 10 600 python3 bench.py --config c4 --res 1024 --spp 8 --steps 1 --warmup 1 > gpurun_out/c4_final.json 2> gpurun_out/c4.err
echo done
