set -eo pipefail
# Round-1 re-entry confirmation on the GPU box: parity tests, smoke, default bench, rocprof.
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
bash tools/profile.sh r01e --steps 1 --warmup 0 --cpu-baseline 0
echo done
