#!/bin/bash
# Fused bounce block size (LUMO_BOUNCE_THREADS): parity at 64 and 128, then C1 at 1024^2 and 362^2.
set -o pipefail
mkdir -p gpurun_out/abf
for t in 64 128; do
  LUMO_BOUNCE_THREADS=$t timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_v$t.log 2>&1
  rc=$?; echo "pytest $t rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_v$t.log | tail -1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for r in 362 1024; do for t in 256 128 64; do
  LUMO_BOUNCE_THREADS=$t timeout -k 10 200 python3 bench.py --res $r --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_${r}_t$t.json
  echo "res $r threads $t $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_${r}_t$t.json'));print(d['value'],d['ms_per_step'])")"
done; done
