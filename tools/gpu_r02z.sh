#!/bin/bash
# Multi-rank bench path rehearsed on one GPU: 2 ranks (gloo, both on device 0), C1 at 512^2.
set -o pipefail
mkdir -p gpurun_out
LUMO_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --res 512 --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err
echo "rc=$?"; cat gpurun_out/bench_2rank.json | head -c 600
