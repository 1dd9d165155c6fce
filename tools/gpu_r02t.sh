#!/bin/bash
# C1 per-rank efficiency at smaller shares (a rank of a 2/4/8-GPU run holds 1/N of the 4 M slots).
set -o pipefail
mkdir -p gpurun_out/abf
for r in 1024 724 512 362; do
  timeout -k 10 200 python3 bench.py --res $r --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/c1_res$r.json
  echo "res $r $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c1_res$r.json'));print(d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['roofline']['stages'].items() if v['ms']>0})")"
done
bash tools/trace_c1.sh r362 --res 362
