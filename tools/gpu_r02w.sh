#!/bin/bash
# Two head streams (LUMO_PIPELINE=2): parity suite, then C1 at 1024^2 / 724^2 / 512^2 / 362^2.
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_w.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_w.log | tail -1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 362 512 724 1024; do for pp in 1 2; do
  LUMO_PIPELINE=$pp timeout -k 10 200 python3 bench.py --res $r --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_${r}_p$pp.json
  echo "res $r pipe $pp $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_${r}_p$pp.json'));print(d['value'],d['ms_per_step'])")"
done; done
