#!/bin/bash
# A/B the device-code variants on the bench workload (run on the GPU box).  Usage: tools/ab.sh v1 v2 ...
# "base" = lumo_amd/liblumo_amd.so.  Each run: 1 warmup + 1 timed step, no CPU baseline.
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=$(pwd)/lumo_amd/liblumo_amd_$v.so; fi
  LUMO_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
done
