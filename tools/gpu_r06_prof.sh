# round-6 rocprofv3 passes (kernel trace + FETCH / WRITE / SQ, tools/profile.sh) of the wide-accel
# workloads: full C3 and C2 frames (PROF_SET=a) or one rank's 1/8 C4 share and C1 (PROF_SET=b)
set -o pipefail
cd $GRAFT_REPO_ROOT
if [ "${PROF_SET:-a}" = "a" ]; then
  bash tools/profile.sh r06_c3 --config c3 --steps 1 --warmup 1 --cpu-baseline 0 &&
  bash tools/profile.sh r06_c2 --config c2 --steps 1 --warmup 1 --cpu-baseline 0
else
  bash tools/profile.sh r06_c4_share --config c4 --spp 4096 --share 0/8 --steps 1 --warmup 1 --cpu-baseline 0 &&
  bash tools/profile.sh r06_c1 --config c1 --steps 1 --warmup 1 --cpu-baseline 0 --bistro-frames 0 --dragon-frames 0 --c4-share=
fi
