# A/B of the accel mode on short frames of every config (bench.py --accel lumo / wide).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r06ab}
mkdir -p $OUT
for cfg in "c2 --spp 4" "c3 --spp 8" "c4 --spp 8" "c1 --spp 64"; do
  set -- $cfg
  for acc in lumo wide; do
    timeout -k 10 300 python -u bench.py --config $1 --spp $3 --steps 2 --warmup 1 --cpu-baseline 0 \
        --bistro-frames 0 --dragon-frames 0 --c4-share "" --accel $acc > $OUT/$1_$acc.json 2> $OUT/$1_$acc.err || exit $?
  done
done
