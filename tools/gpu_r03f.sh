set -eo pipefail
mkdir -p gpurun_out/r03f
REPO=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/r03f/share_trace -o run -- \
  python3 $REPO/bench.py --config c3 --share 0/8 --spp 16 --steps 1 --warmup 1 --cpu-baseline 0 > $REPO/gpurun_out/r03f/share.json 2> $REPO/gpurun_out/r03f/share.err
cd $REPO
echo done
