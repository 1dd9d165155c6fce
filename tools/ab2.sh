#!/bin/bash
# A/B of device-code variants and options on the GPU box (repo root).  Each argument is
# "name[:ENV=val,ENV2=val]" (name = lumo_amd/var/liblumo_amd_<name>.so, "base" = the in-tree
# library); AB_CONFIGS picks short frames of the bench configs (default "c2 c3 c4"), AB_ACCEL the
# accel (default auto).  Results: gpurun_out/${AB_TAG:-ab}/<tag>_<cfg>.json, one line each on stdout.
set -eo pipefail
OUT=gpurun_out/${AB_TAG:-ab}
mkdir -p $OUT
CFGS=${AB_CONFIGS:-c2 c3 c4}
COMMON="--steps 1 --warmup 1 --cpu-baseline 0 --bistro-frames 0 --dragon-frames 0 --c4-share= --accel ${AB_ACCEL:-auto}"
for v in "$@"; do
  name=${v%%:*}; envs=""; [ "$name" != "$v" ] && envs=${v#*:}
  lib=lumo_amd/var/liblumo_amd_${name}.so; [ "$name" = "base" ] && lib=lumo_amd/liblumo_amd.so
  tag=$(echo "$v" | tr ':=,' '___')
  for cfg in $CFGS; do
    case $cfg in
      c1) args="--config c1 --res 1024 --spp 64 --steps 2" ;;
      c1share) args="--config c1 --spp 1024 --share 0/8" ;;
      c2) args="--config c2 --spp 4" ;;
      c4) args="--config c4 --spp 8" ;;
      c4share) args="--config c4 --spp 512 --share 0/8" ;;
      c3share) args="--config c3 --spp 64 --share 0/8" ;;
      *) args="--config c3 --spp 8" ;;
    esac
    env $(echo $envs | tr ',' ' ') LUMO_AMD_LIB=$lib timeout -k 10 300 python3 bench.py $COMMON $args > $OUT/${tag}_${cfg}.json
    python3 -c "import json,sys; d=json.load(open('$OUT/${tag}_${cfg}.json')); st=d['roofline']['stages']; print('$tag $cfg', d['ms_per_step'], 'ms', {k: v['busy_ms'] for k, v in st.items() if v['ms'] > 0})"
  done
done
