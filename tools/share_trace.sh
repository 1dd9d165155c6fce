# usage: bash /tmp/w/tr.sh <outdir> <name> [ENV=val ...]: one share frame under a kernel trace, occupancy summary
set -eo pipefail
R=$(pwd); OUT=$1; NAME=$2; shift 2
mkdir -p $OUT
(cd /tmp && export TMPDIR=/tmp && { [ $# -eq 0 ] || export "$@"; } && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/$NAME \
   -o run -- python3 $R/bench.py --share 0/8 --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 \
   > $R/$OUT/$NAME.json 2> $R/$OUT/$NAME.err)
python3 tools/stream_busy.py $OUT/$NAME/run_kernel_trace.csv > $OUT/${NAME}_busy.json
rm -rf $OUT/$NAME
python3 -c "
import json; d=json.load(open('$OUT/${NAME}_busy.json')); print('$NAME span', round(d['span_ms'],1), 'busy', round(d['busy_ms'],1))
for k,v in list(d['families'].items())[:6]: print('  ', k, v['n'], round(v['sum_ms'],1), round(v['busy_ms'],1), round(v['avg_us'],1))
for k,v in d['queues'].items(): print('  q', k, v['n'], round(v['sum_ms'],1), round(v['busy_ms'],1))
"
