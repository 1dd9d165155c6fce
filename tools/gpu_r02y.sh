#!/bin/bash
# Three head streams (LUMO_PIPELINE=3) vs two: parity, then C1 at 362^2 / 512^2 / 1024^2.
set -o pipefail
mkdir -p gpurun_out/abf
LUMO_PIPELINE=3 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_y.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_y.log | tail -1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 362 512 1024; do for pp in 2 3; do
  LUMO_PIPELINE=$pp timeout -k 10 200 python3 bench.py --res $r --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_${r}_q$pp.json
  echo "res $r pipe $pp $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_${r}_q$pp.json'));print(d['value'],d['ms_per_step'])")"
done; done
