#!/bin/bash
# Deeper PMC view of one workload (run ON the GPU box from the repo root), three passes of their
# own (no traces): lane utilisation / wait / instruction mix, L1->L2 latency and hit rates,
# memory-level parallelism.  Usage: tools/pmc_deep.sh <tag> "<bench args>" [LUMO_AMD_LIB path]
set -eo pipefail
TAG=$1; ARGS="$2"; LIB=${3:-}
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmcd/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -n "$LIB" ] && export LUMO_AMD_LIB=$REPO/$LIB
P=1
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_FLAT SQ_INSTS_VMEM_RD" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_LATENCY_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"; do
  timeout -s KILL 240 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$P -o run -- python3 $REPO/bench.py $ARGS > $OUT/p$P.json 2> $OUT/p$P.err
  P=$((P+1))
done
cd $REPO
python3 tools/pmc_sum.py gpurun_out/pmcd $TAG --all
