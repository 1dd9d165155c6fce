#!/bin/bash
# Quick GPU check (repo root on the GPU box): the parity tests most sensitive to traversal /
# shading changes, then the C1 / C3 A/B of the given variants (tools/ab.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_textures.py tests/test_gpu_materials.py tests/test_gpu_bdpt.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_quick.log | tail -1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab.sh "$@"
