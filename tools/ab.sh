#!/bin/bash
# A/B of device-code variants on the GPU box (repo root): for each "name[:ENV=val,ENV2=val]" argument
# run C1 (1024^2 @ 64 spp, 4 frames), C1 at the bench's own configuration (c1full: 1024^2 @ 1024 spp,
# one frame), C2 (4 spp), C3 (1920x1080 @ 8 spp) and / or C4 (8 spp) with
# lumo_amd/var/liblumo_amd_<name>.so (name "base": the in-tree library).  AB_CONFIGS picks the
# configs (default "c1 c3").  Each run has its own time limit; results: gpurun_out/ab/<tag>_<cfg>.json.
set -eo pipefail
mkdir -p gpurun_out/ab
CFGS=${AB_CONFIGS:-c1 c3}
for v in "$@"; do
  name=${v%%:*}; envs=""; [ "$name" != "$v" ] && envs=${v#*:}
  lib=lumo_amd/var/liblumo_amd_${name}.so; [ "$name" = "base" ] && lib=lumo_amd/liblumo_amd.so
  tag=$(echo "$v" | tr ':=,' '___')
  for cfg in $CFGS; do
    case $cfg in
      c1) args="--res 1024 --spp 64 --steps 4 --warmup 1 --bistro-frames 0 --cpu-baseline 0" ;;
      c1full) args="--steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0" ;;
      c2) args="--config c2 --spp 4 --steps 1 --warmup 1 --cpu-baseline 0" ;;
      c4) args="--config c4 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0" ;;
      *) args="--config c3 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0" ;;
    esac
    env $(echo $envs | tr ',' ' ') LUMO_AMD_LIB=$lib timeout -k 10 300 python3 bench.py $args > gpurun_out/ab/${tag}_${cfg}.json
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/${tag}_${cfg}.json')); st=d['roofline']['stages']; print('$tag $cfg', d['ms_per_step'], 'ms', {k: v['ms'] for k, v in st.items() if v['ms'] > 0})"
  done
done
