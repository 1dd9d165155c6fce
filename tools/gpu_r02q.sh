#!/bin/bash
# C1 dynamic block fetch (LUMO_DYN) and LDS grid cap, at 512^2 (one rank's share of 4 GPUs) and 1024^2.
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_q.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in LUMO_DYN=1 LUMO_DYN=0 LUMO_DYN=1,LUMO_LDS_GRID=768 LUMO_DYN=1,LUMO_LDS_GRID=4096; do
  env $(echo $v | tr ',' ' ') timeout -k 10 200 python3 bench.py --res 512 --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_512_$v.json
  echo "c1_512 $v $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_512_$v.json'));print(d['value'],d['ms_per_step'])")"
done
for v in LUMO_DYN=1 LUMO_DYN=0; do
  env $(echo $v | tr ',' ' ') timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_$v.json
  echo "c1 $v $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_$v.json'));print(d['value'],d['ms_per_step'])")"
done
