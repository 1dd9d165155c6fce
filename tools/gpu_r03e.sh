set -eo pipefail
AB_CONFIGS=c3 bash tools/ab.sh base:LUMO_TOP_GRID=256 base:LUMO_TOP_GRID=256,LUMO_TOP_KB=80 base:LUMO_TOP_GRID=256,LUMO_TOP_KB=120 base:LUMO_TOP_GRID=128
AB_CONFIGS=c2 bash tools/ab.sh base base:LUMO_TOP=0 base:LUMO_TOP_GRID=256
timeout -k 10 600 python3 tools/share_times.py c3 8 64 > gpurun_out/ab/shares_c3_64spp.json
tail -c 700 gpurun_out/ab/shares_c3_64spp.json
echo done
