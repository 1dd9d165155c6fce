#!/bin/bash
# Two-rank rehearsal of the driver's multi-GPU bench on a one-GPU box (gloo, both ranks on GPU 0):
# the static tile % N split and the dynamic shared tile queue, C1 at 64 spp.  Usage:
# tools/gpu_2rank.sh <tag>
set -eo pipefail
OUT=gpurun_out/${1:-2rank}
mkdir -p $OUT
for sch in static dynamic; do
  LUMO_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --res 1024 --spp 64 --steps 2 --warmup 1 \
    --bistro-frames 0 --cpu-baseline 0 --schedule $sch > $OUT/bench_2rank_$sch.json 2> $OUT/bench_2rank_$sch.err
  head -c 400 $OUT/bench_2rank_$sch.json; echo
done
