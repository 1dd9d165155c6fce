#!/bin/bash
# C4 (caustics BDPT, 1024^2 @ 8 spp) A/B of device-code variants (repo root on the GPU box).
set -eo pipefail
mkdir -p gpurun_out/ab
for v in "$@"; do
  lib=lumo_amd/var/liblumo_amd_${v}.so; [ "$v" = "base" ] && lib=lumo_amd/liblumo_amd.so
  LUMO_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --config c4 --res 1024 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/ab/${v}_c4.json
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab/${v}_c4.json')); st=d['roofline']['stages']
print('${v}', d['msamples_per_s'], 'Msamples/s', d['ms_per_step'], 'ms', {k: round(v['ms'],1) for k, v in st.items() if v['ms']})"
done
