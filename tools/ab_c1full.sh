#!/bin/bash
# A/B at the bench's own C1 configuration (1024^2 @ 1024 spp, one step after one warmup step):
# for each "name[:ENV=val,...]" argument (name "base" = the in-tree library, else
# lumo_amd/var/liblumo_amd_<name>.so).  Results: gpurun_out/abf/<tag>.json.
set -eo pipefail
mkdir -p gpurun_out/abf
for v in "$@"; do
  name=${v%%:*}; envs=""; [ "$name" != "$v" ] && envs=${v#*:}
  lib=lumo_amd/var/liblumo_amd_${name}.so; [ "$name" = "base" ] && lib=lumo_amd/liblumo_amd.so
  tag=$(echo "$v" | tr ':=,' '___')
  env $(echo $envs | tr ',' ' ') LUMO_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/abf/${tag}.json
  echo "$tag $(python3 -c "import json;d=json.load(open('gpurun_out/abf/${tag}.json'));print(d['value'],d['ms_per_step'])")"
done
