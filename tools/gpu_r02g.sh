#!/bin/bash
# Fused bounce kernel: parity (Cornell, all bounce modes) then the C1 A/B at the bench config.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_materials.py tests/test_gpu_scenes.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_g.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_g.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_c1full.sh base:LUMO_FUSED=0 base base:LUMO_TAIL=0 base:LUMO_TAIL=262144 base:LUMO_TAIL=16384 w2 w2:LUMO_TAIL=262144
