#!/bin/bash
# One GPU-box pass (run from the repo root via gpurun): GPU parity tests, smoke, default bench,
# then the rocprofv3 kernel-trace + FETCH_SIZE + WRITE_SIZE passes of a 1-step bench.
# Every GPU step has its own time limit; the first failure ends the script.
set -eo pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
if [ "${PROFILE:-1}" = "1" ]; then
  bash tools/profile.sh $TAG --steps 1 --warmup 0 --cpu-baseline 0
fi
echo done
