set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/ab
bash tools/ab.sh base r01 w5 w6 w8
