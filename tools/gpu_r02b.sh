#!/bin/bash
# Round-2 GPU pass B (repo root on the GPU box): texture parity first, then every GPU test,
# smoke, and the shade-waves A/B (base vs SHADE_WAVES=2 vs the round-1 tree) on C1 / C3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_textures.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_tex.log 2>&1
rc=$?; echo "tex rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --ignore tests/test_gpu_textures.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
bash tools/ab.sh base sh2 r01
echo done
