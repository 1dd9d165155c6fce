#!/bin/bash
# Execution-knob sweep at one rank's 1/8 share of C1 (1024² @ 1024 spp, tile % 8 == 0) on one GPU.
# Arguments: "name[:ENV=val,ENV2=val]" ("base" = defaults).  Results: gpurun_out/<tag>/share_<name>.json
set -eo pipefail
OUT=gpurun_out/${SWEEP_TAG:-share_sweep}
mkdir -p $OUT
for v in "$@"; do
  name=${v%%:*}; envs=""; [ "$name" != "$v" ] && envs=${v#*:}
  tag=$(echo "$v" | tr ':=,' '___')
  env $(echo $envs | tr ',' ' ') timeout -k 10 200 python3 bench.py --share 0/8 --steps 3 --warmup 1 \
    --bistro-frames 0 --cpu-baseline 0 > $OUT/share_$tag.json 2> $OUT/share_$tag.err
  python3 -c "import json; d=json.load(open('$OUT/share_$tag.json')); print('$v', d['ms_per_step'], 'ms')"
done
