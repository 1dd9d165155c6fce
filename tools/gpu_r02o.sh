#!/bin/bash
# Nearest-first visibility walks: full GPU suite; C1 and C3 A/B against lumo's order (variant nv0).
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_o.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_o.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_c1full.sh base nv0
for v in base nv0; do
  lib=lumo_amd/var/liblumo_amd_$v.so; [ $v = base ] && lib=lumo_amd/liblumo_amd.so
  LUMO_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --config c3 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/abf/c3_$v.json
  echo "c3_$v $(python3 -c "import json;d=json.load(open('gpurun_out/abf/c3_$v.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],{k:v['ms'] for k,v in r['stages'].items() if v['ms']>0},r['per_query'])")"
done
