#!/bin/bash
# Collect one set of PMC counters (own pass, no traces) for the bench command; run on the GPU box.
# Usage: tools/pmc.sh <tag> "<COUNTERS...>" [bench args...]
set -e
TAG=$1; CTRS=$2; shift 2
REPO=$(pwd); OUT=$REPO/gpurun_out/pmc/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc $CTRS --output-format csv -d $OUT -o run -- python3 $REPO/bench.py "$@" > $OUT/bench.json 2> $OUT/err.txt
