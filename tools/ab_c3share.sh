#!/bin/bash
# C3 at one rank's 1/8 share and the full frame (64 spp each), for each library tag given
# ("base": the in-tree library, else lumo_amd/var/liblumo_amd_<tag>.so); results in gpurun_out/$OUT.
set -eo pipefail
OUT=gpurun_out/${AB_OUT:-ab_c3share}
mkdir -p $OUT
for v in "$@"; do
  lib=lumo_amd/var/liblumo_amd_${v}.so; [ "$v" = "base" ] && lib=lumo_amd/liblumo_amd.so
  LUMO_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --config c3 --spp 64 --share 0/8 --steps 1 --warmup 1 --cpu-baseline 0 > $OUT/${v}_share.json
  LUMO_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --config c3 --spp 64 --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/${v}_full.json
  python3 -c "import json; s=json.load(open('$OUT/${v}_share.json')); f=json.load(open('$OUT/${v}_full.json')); print('$v share', s['ms_per_step'], 'full', f['ms_per_step'], 'share rate', round(f['ms_per_step']/8/s['ms_per_step'],3))"
done
