#!/bin/bash
# PMC comparison of device-code variants on one workload (run ON the GPU box from the repo root):
# for each variant name (base = in-tree library, r01 = the round-1 tree, else lumo_amd/var/...):
#   pass A: SQ waves / instruction mix / wave cycles / wait cycles (8 SQ counters)
#   pass B: L2 hits / misses, HBM read / write requests
# each pass in its own rocprofv3 run, never combined with traces.  Summaries: tools/pmc_sum.py.
# Usage: tools/pmc_cmp.sh "<bench args>" name...
set -eo pipefail
ARGS="$1"; shift
REPO=$(pwd)
for v in "$@"; do
  lib=$REPO/lumo_amd/var/liblumo_amd_$v.so; bench=$REPO/bench.py
  [ "$v" = "base" ] && lib=$REPO/lumo_amd/liblumo_amd.so
  if [ "$v" = "r01" ]; then lib=$REPO/ab_r01/lumo_amd/liblumo_amd.so; bench=$REPO/ab_r01/bench.py; fi
  OUT=$REPO/gpurun_out/pmc/$v
  mkdir -p $OUT
  cd /tmp && export TMPDIR=/tmp
  export LUMO_AMD_LIB=$lib
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/a -o run -- python3 $bench $ARGS > $OUT/a.json 2> $OUT/a.err
  timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $OUT/b -o run -- python3 $bench $ARGS > $OUT/b.json 2> $OUT/b.err
  unset LUMO_AMD_LIB
  cd $REPO
done
python3 tools/pmc_sum.py gpurun_out/pmc "$@"
