#!/bin/bash
# Pipelined passes: fused head bounces per pass (LUMO_HEADS) at 1024^2 and 362^2; parity at 4 and 8.
set -o pipefail
mkdir -p gpurun_out/abf
for h in 4 8; do
  LUMO_HEADS=$h timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_h$h.log 2>&1
  rc=$?; echo "pytest heads $h rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_h$h.log | tail -1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for r in 1024 362; do for h in 5 6 7 8; do
  LUMO_HEADS=$h timeout -k 10 200 python3 bench.py --res $r --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_${r}_h$h.json
  echo "res $r heads $h $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_${r}_h$h.json'));print(d['value'],d['ms_per_step'])")"
done; done
