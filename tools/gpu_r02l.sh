#!/bin/bash
# Film terms precomputed per sample: parity (film / tile tests), then C1 A/B of tail threshold and bounce-ahead.
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_textures.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_l.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_l.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_c1full.sh base base:LUMO_TAIL=65536 base:LUMO_TAIL=1048576 base:LUMO_BOUNCE_AHEAD=2 base:LUMO_BOUNCE_AHEAD=5
