#!/bin/bash
# Pipelined passes: full GPU suite; C1 pipeline on/off at the bench config and at 512^2 (a quarter of
# the slots, as one rank of a 4-GPU run has).
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_p.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_p.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_c1full.sh base base:LUMO_PIPELINE=0
for v in LUMO_PIPELINE=1 LUMO_PIPELINE=0; do
  env $v timeout -k 10 200 python3 bench.py --res 512 --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_512_$v.json
  echo "c1_512 $v $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_512_$v.json'));print(d['value'],d['ms_per_step'])")"
done
