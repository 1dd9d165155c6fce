#!/bin/bash
# A/B over "variant:ENV=VAL" specs.  base = default library.
for spec in "$@"; do
  v=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
  if [ "$v" = base ]; then lib=""; else lib=$(pwd)/lumo_amd/liblumo_amd_$v.so; fi
  name=$(echo "$spec" | tr ':=,' '___')
  env $(echo $envs | tr ',' ' ') LUMO_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || exit 1
done
