#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_h5.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_h5.log | tail -1
