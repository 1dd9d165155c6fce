#!/bin/bash
# One bench configuration under several environment settings: ab_env.sh "<bench args>" tag:ENV=v,ENV2=w ...
# (tag "base": no extra environment); results gpurun_out/${AB_OUT:-ab_env}/<tag>.json, one summary line each.
set -eo pipefail
OUT=gpurun_out/${AB_OUT:-ab_env}
mkdir -p $OUT
ARGS=$1; shift
for v in "$@"; do
  tag=${v%%:*}; envs=""; [ "$tag" != "$v" ] && envs=${v#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 300 python3 bench.py $ARGS --cpu-baseline 0 > $OUT/$tag.json
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); st=d['roofline']['stages']; print('$tag', d['ms_per_step'], 'ms', {k: v['busy_ms'] for k, v in st.items() if v['ms'] > 0})"
done
