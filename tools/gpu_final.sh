#!/bin/bash
# End-of-session check of the committed tree: full GPU suite, smoke, default bench line.
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo done
