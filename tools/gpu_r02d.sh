#!/bin/bash
# Round-2 GPU pass D (repo root on the GPU box): rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE
# passes of C1 (1024^2 @ 256 spp) and C3 (Bistro @ 8 spp), for profiles/r02 and pmc_traffic.json.
set -eo pipefail
bash tools/profile.sh r02_c1 --config c1 --spp 256 --steps 1 --warmup 0 --cpu-baseline 0 --bistro-frames 0
bash tools/profile.sh r02_c3 --config c3 --spp 8 --steps 1 --warmup 0 --cpu-baseline 0
echo done
