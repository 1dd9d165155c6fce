#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for 8-B-per-lane streams (GPU box, repo root).
set -e
REPO=$(pwd); OUT=$REPO/gpurun_out/calib; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $REPO/tools/calib.py > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $REPO/tools/calib.py > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $REPO/tools/calib.py > $OUT/write.log 2>&1
cd $REPO && python3 tools/parse_prof.py $OUT > $OUT/summary.json
