#!/bin/bash
# C1 at 362^2 (one rank's share of 8 GPUs): grid cap and pipeline probes.
set -o pipefail
mkdir -p gpurun_out/abf
for v in LUMO_X=0 LUMO_LDS_GRID=768 LUMO_LDS_GRID=512 LUMO_LDS_GRID=1024 LUMO_LDS_GRID=4096 LUMO_PIPELINE=0 LUMO_DYN=0; do
  env $v timeout -k 10 200 python3 bench.py --res 362 --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_362_$v.json
  echo "362 $v $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_362_$v.json'));print(d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['roofline']['stages'].items() if v['ms']>0})")"
done
