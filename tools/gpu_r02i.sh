#!/bin/bash
# Per-block queue grouping (LUMO_QSORT): parity with it on, then C1 (bench config) and C3 (8 spp) A/B.
set -o pipefail
mkdir -p gpurun_out/abf
LUMO_QSORT=3 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenes.py tests/test_gpu_materials.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_i.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_i.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_c1full.sh base base:LUMO_QSORT=1 base:LUMO_QSORT=2 base:LUMO_QSORT=3
for q in 0 3 1; do
  LUMO_QSORT=$q timeout -k 10 300 python3 bench.py --config c3 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/abf/c3_q$q.json
  echo "c3 q$q $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c3_q$q.json'));print(d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['roofline']['stages'].items() if v['ms']>0})")"
done
