set -eo pipefail
mkdir -p gpurun_out
bash tools/ab.sh c5 c6 base
echo ok
