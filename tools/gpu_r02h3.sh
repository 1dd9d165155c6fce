#!/bin/bash
# Auto head count (RR bounce to the tail kernel below 2 M slots) + set-reuse wait in every mode:
# parity at heads 4 / auto, full suite; C1 at 1024 / 724 / 512 / 362.
set -o pipefail
mkdir -p gpurun_out/abf
LUMO_HEADS=4 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_h4.log 2>&1
rc=$?; echo "pytest heads 4 rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_h4.log | tail -1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1024 724 512 362; do
  timeout -k 10 200 python3 bench.py --res $r --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_${r}_auto.json
  echo "res $r auto $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_${r}_auto.json'));print(d['value'],d['ms_per_step'])")"
done
LUMO_HEADS=6 timeout -k 10 200 python3 bench.py --res 512 --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_512_h6.json
echo "res 512 heads 6 $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_512_h6.json'));print(d['value'],d['ms_per_step'])")"
