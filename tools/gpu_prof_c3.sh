# rocprofv3 kernel trace + SQ counters of C3 at 8 spp in both accel modes (tools/profile.sh passes 1 and 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
REPO=$(pwd)
for acc in lumo wide; do
  OUT=$REPO/gpurun_out/${TAG:-r06p}/c3_$acc
  mkdir -p $OUT
  ARGS="--config ${CFG:-c3} --spp ${SPP:-8} --steps 1 --warmup 1 --cpu-baseline 0 --bistro-frames 0 --dragon-frames 0 --c4-share= --accel $acc"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $REPO/bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err) || exit $?
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_FLAT SQ_INSTS_LDS \
    --output-format csv -d $OUT/valu -o run -- python3 $REPO/bench.py $ARGS > $OUT/bench_valu.json 2> $OUT/valu.err) || exit $?
  python3 tools/parse_prof.py $OUT > $OUT/summary.json || exit $?
  find $OUT -name '*.csv' ! -name 'run_kernel_stats.csv' -delete
done
