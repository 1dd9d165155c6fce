#!/bin/bash
# Two-rank rehearsal of the driver's multi-GPU bench on a one-GPU box (gloo, both ranks on GPU 0),
# C1 at 64 spp, per schedule argument: "static" (tile % N), "dynamic" (shared TileQueue, default
# chunk) or "dynamic:<tiles per claim>".  Usage: tools/gpu_2rank.sh <tag> [schedule ...]
set -eo pipefail
OUT=gpurun_out/${1:-2rank}
shift || true
mkdir -p $OUT
for spec in ${@:-static dynamic}; do
  sch=${spec%%:*}; extra=""
  [ "$sch" != "$spec" ] && extra="--chunk ${spec#*:}"
  tag=$(echo $spec | tr ':' '_')
  LUMO_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --res 1024 --spp 64 --steps 2 --warmup 1 \
    --bistro-frames 0 --cpu-baseline 0 --schedule $sch $extra > $OUT/bench_2rank_$tag.json 2> $OUT/bench_2rank_$tag.err
  python3 -c "import json; d=json.loads([l for l in open('$OUT/bench_2rank_$tag.json') if l.startswith('{')][-1]); print('$spec', d['ms_per_step'], 'ms', d['value'], 'Mrays/s')"
done
