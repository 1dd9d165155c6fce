set -eo pipefail
mkdir -p gpurun_out/r03g gpurun_out/ab
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03g/pytest.log 2>&1 || { tail -40 gpurun_out/r03g/pytest.log; exit 1; }
tail -1 gpurun_out/r03g/pytest.log
AB_CONFIGS=c3 bash tools/ab.sh base base:LUMO_SPLIT_GROUPS=1 base:LUMO_SPLIT_GROUPS=4
LUMO_SPLIT_PIPE=4 timeout -k 10 600 python3 tools/share_times.py c3 8 64 > gpurun_out/ab/shares_c3_64spp_k4.json
tail -c 300 gpurun_out/ab/shares_c3_64spp_k4.json
echo done
