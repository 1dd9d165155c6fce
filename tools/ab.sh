#!/bin/bash
# A/B of device-code variants on the GPU box (repo root): for each "name[:ENV=val]" argument run
# C1 (1024^2 @ 64 spp, 4 frames) and C3 (1920x1080 @ 8 spp) with lumo_amd/var/liblumo_amd_<name>.so
# (name "base": the in-tree library; "r01": the round-1 tree copied to ab_r01/).  Results: gpurun_out/ab/<name>_<cfg>.json.
set -eo pipefail
mkdir -p gpurun_out/ab
for v in "$@"; do
  name=${v%%:*}; envs=""; [ "$name" != "$v" ] && envs=${v#*:}
  lib=lumo_amd/var/liblumo_amd_${name}.so; [ "$name" = "base" ] && lib=lumo_amd/liblumo_amd.so
  tag=$(echo "$v" | tr ':=,' '___')
  bench="bench.py"; extra="--bistro-frames 0"
  if [ "$name" = "r01" ]; then bench="ab_r01/bench.py"; extra=""; lib=ab_r01/lumo_amd/liblumo_amd.so; fi  # round-1 tree
  env $(echo $envs | tr ',' ' ') LUMO_AMD_LIB=$lib timeout -k 10 300 python3 $bench --res 1024 --spp 64 --steps 4 --warmup 1 $extra --cpu-baseline 0 > gpurun_out/ab/${tag}_c1.json
  env $(echo $envs | tr ',' ' ') LUMO_AMD_LIB=$lib timeout -k 10 300 python3 $bench --config c3 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/ab/${tag}_c3.json
done
python3 tools/ab_report.py
