#!/bin/bash
# Phased fused bounce (LUMO_FUSED=1) vs three kernels, both with the tail kernel; parity first.
set -o pipefail
mkdir -p gpurun_out/abf
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_j.log | tail -3; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_c1full.sh base base:LUMO_FUSED=1 w2:LUMO_FUSED=1 base
