#!/bin/bash
# Round-2 GPU pass F (repo root on the GPU box), after the while-while traversal loops:
# full GPU parity suite, smoke, the default bench line (C1 + C3 @256 spp), then rocprofv3 traces +
# FETCH/WRITE passes of C1 (256 spp) and C3 (8 spp).
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
bash tools/profile.sh c1 --spp 256 --steps 1 --warmup 0 --bistro-frames 0 --cpu-baseline 0
bash tools/profile.sh c3 --config c3 --spp 8 --steps 1 --warmup 0 --cpu-baseline 0
echo done
