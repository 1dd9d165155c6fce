#!/bin/bash
# Default = two head streams: full GPU suite, smoke, C1 at 1024^2 and 362^2.
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_x.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_x.log | tail -1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; tail -1 gpurun_out/smoke.log
for r in 362 1024; do
  timeout -k 10 200 python3 bench.py --res $r --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_${r}_p2b.json
  echo "res $r $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_${r}_p2b.json'));print(d['value'],d['ms_per_step'],d['queries_per_step'])")"
done
