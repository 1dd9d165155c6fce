set -eo pipefail
mkdir -p gpurun_out/r03d
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_trace.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d/pytest.log 2>&1 || { tail -40 gpurun_out/r03d/pytest.log; exit 1; }
tail -1 gpurun_out/r03d/pytest.log
AB_CONFIGS=c3 bash tools/ab.sh base base:LUMO_TOP=0 base:LUMO_TOP_GRID=256 base:LUMO_TOP_GRID=512
echo done
