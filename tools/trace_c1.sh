#!/bin/bash
# rocprofv3 kernel trace of C1 with extra bench arguments; output gpurun_out/prof/c1_<tag>/.
set -eo pipefail
R=$(pwd)
tag=$1; shift
mkdir -p $R/gpurun_out/prof/c1_$tag
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof/c1_$tag/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 "$@" > $R/gpurun_out/prof/c1_$tag/bench.json 2> $R/gpurun_out/prof/c1_$tag/err.txt
