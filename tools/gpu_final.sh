#!/bin/bash
# Check of the tree on the GPU box (repo root): full GPU suite, smoke, default bench line, then
# (optional, "trace") a rocprofv3 kernel trace of one C1 frame.  Every GPU step has its own time
# limit and the chain stops at the first failure.  Usage: tools/gpu_final.sh <tag> [trace]
set -eo pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
head -c 600 $OUT/bench.json; echo
if [ "${2:-}" = "trace" ]; then
  REPO=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/trace -o run -- \
    python3 $REPO/bench.py --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > $REPO/$OUT/bench_trace.json 2> $REPO/$OUT/trace.err
  cd $REPO
fi
echo done
