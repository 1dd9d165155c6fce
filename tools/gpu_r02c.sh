#!/bin/bash
# Round-2 GPU pass C (repo root on the GPU box): every GPU test, smoke, the default bench
# (C1 Cornell 1024^2 @ 1024 spp + C3 Bistro stand-in 1920x1080 @ 256 spp).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 900 python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
