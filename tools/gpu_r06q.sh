# C3 1/8 share against the full frame at 64 spp (per-slot rate), wide accel (bench auto)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06q
for run in full share full share; do
  if [ $run = full ]; then a="--config c3 --spp 64"; else a="--config c3 --spp 64 --share 0/8"; fi
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 $a > gpurun_out/r06q/c3_$run.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r06q/c3_$run.json')); print('$run', d['ms_per_step'])"
done
