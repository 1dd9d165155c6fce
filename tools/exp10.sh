set -eo pipefail
mkdir -p gpurun_out/prof/c4
REPO=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/prof/c4/trace -o run -- python3 $REPO/bench.py --config c4 --res 1024 --spp 4 --steps 1 --warmup 0 --cpu-baseline 0 > $REPO/gpurun_out/prof/c4/bench.json 2> $REPO/gpurun_out/prof/c4/err.txt
echo ok
