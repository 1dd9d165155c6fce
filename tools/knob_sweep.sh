#!/bin/bash
# C1 full frame (2 timed frames) and one rank's 1/8 share (3 timed frames) per execution-knob set,
# on one GPU.  Arguments: "name[:ENV=val,ENV2=val]" ("base" = defaults); MODE=full|share|both.
# Results: gpurun_out/<SWEEP_TAG>/{full,share}_<name>.json and one summary line per run.
set -eo pipefail
OUT=gpurun_out/${SWEEP_TAG:-knob_sweep}
MODE=${MODE:-both}
mkdir -p $OUT
for v in "$@"; do
  name=${v%%:*}; envs=""; [ "$name" != "$v" ] && envs=${v#*:}
  if [ "$MODE" != share ]; then
    env $(echo $envs | tr ',' ' ') timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --bistro-frames 0 \
      --cpu-baseline 0 > $OUT/full_$name.json 2> $OUT/full_$name.err
    python3 -c "import json; d=json.load(open('$OUT/full_$name.json')); print('full $v', d['ms_per_step'], 'ms')"
  fi
  if [ "$MODE" != full ]; then
    env $(echo $envs | tr ',' ' ') timeout -k 10 200 python3 bench.py --share 0/8 --steps 3 --warmup 1 \
      --bistro-frames 0 --cpu-baseline 0 > $OUT/share_$name.json 2> $OUT/share_$name.err
    python3 -c "import json; d=json.load(open('$OUT/share_$name.json')); print('share $v', d['ms_per_step'], 'ms')"
  fi
done
