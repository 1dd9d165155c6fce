set -eo pipefail
mkdir -p gpurun_out/ab
LUMO_SPLIT_GROUPS=4 timeout -k 10 600 python3 tools/share_times.py c3 8 64 > gpurun_out/ab/shares_c3_64spp_g4.json
tail -c 200 gpurun_out/ab/shares_c3_64spp_g4.json; echo
timeout -k 10 600 python3 tools/share_times.py c1 8 64 > gpurun_out/ab/shares_c1_64spp.json
tail -c 200 gpurun_out/ab/shares_c1_64spp.json; echo
echo done
