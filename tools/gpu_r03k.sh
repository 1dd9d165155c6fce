set -eo pipefail
mkdir -p gpurun_out/ab gpurun_out/r03k
LUMO_KD_LDS=8 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_trace.py -m gpu -q -x --timeout 300 --timeout-method thread -k "top or trace or full_scale or split or variants" > gpurun_out/r03k/pytest_kdlds.log 2>&1 || { tail -30 gpurun_out/r03k/pytest_kdlds.log; exit 1; }
tail -1 gpurun_out/r03k/pytest_kdlds.log
AB_CONFIGS=c2 bash tools/ab.sh base base:LUMO_KD_LDS=4 base:LUMO_KD_LDS=8 base:LUMO_KD_LDS=12
AB_CONFIGS=c3 bash tools/ab.sh base:LUMO_KD_LDS=4,LUMO_TOP_KB=100 base:LUMO_KD_LDS=8,LUMO_TOP_KB=64
for v in "LUMO_FUSED_SPLIT=0" "LUMO_FUSED_SPLIT=1"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 600 python3 tools/share_times.py c1 8 256 > gpurun_out/ab/shares_c1_256_$tag.json
  echo "$v"; tail -c 230 gpurun_out/ab/shares_c1_256_$tag.json; echo
done
echo done
