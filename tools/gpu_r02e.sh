#!/bin/bash
# Round-2 GPU pass E (repo root on the GPU box): shadow-waves A/B (base vs 3 waves/SIMD) on C1 / C3,
# then builder measurements of C2 (dragon stand-in, 4 spp) and C4 (caustics BDPT, 8 spp).
set -eo pipefail
mkdir -p gpurun_out
bash tools/ab.sh base w3
timeout -k 10 400 python3 bench.py --config c2 --spp 4 --steps 1 --warmup 1 --cpu-baseline 1 --cpu-seconds 6 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
timeout -k 10 400 python3 bench.py --config c4 --res 1024 --spp 8 --steps 1 --warmup 1 --cpu-baseline 1 --cpu-seconds 6 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
echo done
