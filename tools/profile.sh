#!/bin/bash
# rocprofv3 profile of the bench command (run ON the GPU box from the repo root):
#   1. --kernel-trace --stats          per-kernel launch counts / average durations
#   2. --pmc FETCH_SIZE  (own pass)    HBM read bytes per dispatch
#   3. --pmc WRITE_SIZE  (own pass)    HBM write bytes per dispatch
#   4. --pmc SQ_* VALU / wave counters (own pass)
# PMC passes never combine with sys/runtime/hip traces.  Outputs under gpurun_out/prof/.
# Usage: tools/profile.sh <tag> [bench args...]
set -eo pipefail
TAG=${1:-r01}; shift || true
REPO=$(pwd)
OUT=$REPO/gpurun_out/prof/$TAG
mkdir -p $OUT
ARGS="$@"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $REPO/bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $REPO/bench.py $ARGS > $OUT/bench_fetch.json 2> $OUT/fetch.err
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $REPO/bench.py $ARGS > $OUT/bench_write.json 2> $OUT/write.err
# SQ pass: VALU instructions, lane activity (THREAD_CYCLES / ACTIVE_INST = lanes active per VALU
# instruction), wave cycles and waits, FLAT (incl. scratch) and LDS instructions (8 SQ counters)
timeout -s KILL 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_FLAT SQ_INSTS_LDS \
  --output-format csv -d $OUT/valu -o run -- python3 $REPO/bench.py $ARGS > $OUT/bench_valu.json 2> $OUT/valu.err
cd $REPO && python3 tools/parse_prof.py $OUT > $OUT/summary.json
# keep the summaries (the per-dispatch CSVs of a long run exceed what a gpurun call copies back)
if [ -z "$KEEP_CSV" ]; then
  find $OUT -name '*.csv' ! -name 'run_kernel_stats.csv' -delete
fi
