#!/bin/bash
# Full GPU suite; C1 default (fused + tail) vs three kernels; C2 (dragon, 4 spp) tail / fused A/B.
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_k.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_k.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_c1full.sh base base:LUMO_FUSED=0
for v in "" LUMO_TAIL=0 LUMO_FUSED=1; do
  tag=c2_${v:-base}
  env $v timeout -k 10 300 python3 bench.py --config c2 --spp 4 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/abf/$tag.json
  echo "$tag $(python3 -c "import json;d=json.load(open('gpurun_out/abf/$tag.json'));print(d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['roofline']['stages'].items() if v['ms']>0})")"
done
