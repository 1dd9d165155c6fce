#!/bin/bash
# Per-wave dynamic fetch in closest / shadow / tail kernels: full GPU suite; C1, C1@512, C2, C3.
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_r.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run() { tag=$1; shift; timeout -k 10 300 python3 bench.py "$@" --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/abf/$tag.json; echo "$tag $(python3 -c "import json;d=json.load(open('gpurun_out/abf/$tag.json'));print(d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['roofline']['stages'].items() if v['ms']>0})")"; }
run c1_wf --bistro-frames 0
run c1_512_wf --res 512 --bistro-frames 0
run c2_wf --config c2 --spp 4
run c3_wf --config c3 --spp 8
