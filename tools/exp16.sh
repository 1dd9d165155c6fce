set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trace.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pad.log 2>&1
bash tools/ab.sh base nopad base nopad
echo ok
