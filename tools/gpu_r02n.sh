#!/bin/bash
# Sorted NEE (n_shadow > 1) + tail heuristic: full GPU suite; C1 A/B; C3 A/B of NEE order.
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_n.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_n.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_c1full.sh base
for v in LUMO_NEE_SORT=1 LUMO_NEE_SORT=0 LUMO_BUCKETS=0,LUMO_NEE_SORT=0; do
  tag=c3_$v
  env $(echo $v | tr ',' ' ') timeout -k 10 300 python3 bench.py --config c3 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/abf/$tag.json
  echo "$tag $(python3 -c "import json;d=json.load(open('gpurun_out/abf/$tag.json'));print(d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['roofline']['stages'].items() if v['ms']>0})")"
done
