#!/bin/bash
# One GPU call that checks and measures the tree: the GPU test suite, the C1 line (3 frames), one C3
# frame, C2 at 4 spp, C4 at 8 spp, the fused kernel's phase clocks (diagnostics build, if built), one C1 1/8-share frame set
# and its kernel-trace occupancy; with MEASURE_DEFAULT=1 also the default bench line (C1 + C3 + CPU baselines).  Every step has its own time limit; the chain stops at the first
# failure.  Usage (on the GPU box, repo root): bash tools/measure.sh <tag>
set -o pipefail
TAG=${1:-measure}
OUT=gpurun_out/$TAG
mkdir -p $OUT
R=$(pwd)
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 &&
tail -2 $OUT/pytest.log &&
timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > $OUT/c1.json 2> $OUT/c1.err &&
{ [ -z "$MEASURE_DEFAULT" ] || timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err; } &&
timeout -k 10 200 python3 bench.py --config c3 --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/c3.json 2> $OUT/c3.err &&
timeout -k 10 200 python3 bench.py --config c2 --spp 4 --steps 2 --warmup 1 --cpu-baseline 0 > $OUT/c2.json 2> $OUT/c2.err &&
timeout -k 10 200 python3 bench.py --config c4 --spp 8 --steps 1 --warmup 1 --cpu-baseline 0 > $OUT/c4.json 2> $OUT/c4.err &&
SWEEP_TAG=$TAG timeout -k 10 300 bash tools/share_sweep.sh base &&
{ [ ! -f lumo_amd/var/liblumo_amd_phase.so ] ||
  LUMO_AMD_LIB=lumo_amd/var/liblumo_amd_phase.so timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 \
    --bistro-frames 0 --cpu-baseline 0 > $OUT/phase_full.json 2> $OUT/phase_full.err; } &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/share_trace \
   -o run -- python3 $R/bench.py --share 0/8 --steps 1 --warmup 1 --bistro-frames 0 --cpu-baseline 0 \
   > $R/$OUT/share_trace.json 2> $R/$OUT/share_trace.err) &&
python3 tools/stream_busy.py $OUT/share_trace/run_kernel_trace.csv > $OUT/share_busy.json &&
rm -rf $OUT/share_trace &&
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
for n in ("c1", "c3", "c2", "c4"):
    d = json.load(open(f"{o}/{n}.json"))
    r = d["roofline"]
    print(n, d["value"], d["unit"], d["ms_per_step"], "ms", "frac", r.get("frac"), "stages",
          {k: round(v["busy_ms"], 1) for k, v in r.get("stages", {}).items() if v["busy_ms"]})
b = json.load(open(f"{o}/share_busy.json"))
print("share span", round(b["span_ms"], 1), {k: round(v["busy_ms"], 1) for k, v in b["queues"].items()},
      {k: (v["n"], round(v["avg_us"], 1)) for k, v in list(b["families"].items())[:6]})
PY
