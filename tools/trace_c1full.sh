#!/bin/bash
# rocprofv3 kernel trace of the bench's C1 configuration (1 step after 1 warmup step), optional
# environment assignments as arguments; output gpurun_out/prof/c1full_<tag>/.
set -eo pipefail
R=$(pwd)
tag=$(echo "${*:-base}" | tr ' =' '__')
mkdir -p $R/gpurun_out/prof/c1full_$tag
cd /tmp && export TMPDIR=/tmp
export "$@" 2>/dev/null || true
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof/c1full_$tag/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > $R/gpurun_out/prof/c1full_$tag/bench.json 2> $R/gpurun_out/prof/c1full_$tag/err.txt
