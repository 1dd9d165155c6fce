#!/bin/bash
# A/B only (repo root on the GPU box): tools/ab.sh over the given variants (name[:ENV=val]).
set -eo pipefail
mkdir -p gpurun_out
bash tools/ab.sh "$@"
