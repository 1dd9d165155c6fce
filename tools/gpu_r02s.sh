#!/bin/bash
# Round-2 final-build pass: full GPU suite, smoke, default bench line (C1 + C3 @256 spp),
# rocprofv3 traces + FETCH/WRITE of C1 (bench config) and C3 (8 spp), C2 / C4 builder lines.
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
bash tools/profile.sh c1 --steps 1 --warmup 0 --bistro-frames 0 --cpu-baseline 0
bash tools/profile.sh c3 --config c3 --spp 8 --steps 1 --warmup 0 --cpu-baseline 0
timeout -k 10 400 python3 bench.py --config c2 --spp 4 --steps 1 --warmup 1 --cpu-baseline 1 --cpu-seconds 6 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
echo done
