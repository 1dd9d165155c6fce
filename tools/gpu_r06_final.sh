# round-6 final check: GPU suite, smoke, default bench line (tools/gpu_final.sh) into gpurun_out/r06f
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_final.sh r06f
