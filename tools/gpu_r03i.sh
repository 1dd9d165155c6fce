set -eo pipefail
for i in 1 2 3; do
timeout -k 10 300 python3 tools/debug/tail_mode.py 0 1073741824 0 2>&1 | head -3
timeout -k 10 300 python3 tools/debug/tail_mode.py 1 1073741824 0 2>&1 | head -3
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03g/pytest2.log 2>&1 || true
tail -3 gpurun_out/r03g/pytest2.log
