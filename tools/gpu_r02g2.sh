#!/bin/bash
# C1 (bench config) LDS grid cap with three head streams.
set -o pipefail
mkdir -p gpurun_out/abf
for v in LUMO_X=0 LUMO_LDS_GRID=1024 LUMO_LDS_GRID=4096 LUMO_LDS_GRID=768; do
  env $v timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_g_$v.json
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_g_$v.json'));print(d['value'],d['ms_per_step'])")"
done
