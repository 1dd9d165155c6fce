"""Summarise an A/B run (tools/ab.sh): one line per (variant, workload) JSON in gpurun_out/ab/."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
for p in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        r = json.load(open(p))
    except ValueError:
        print(os.path.basename(p), "(no result)")
        continue
    f = r["roofline"]
    st = " ".join(f"{k}={v['ms']:.0f}" for k, v in f["stages"].items() if v["ms"])
    print(f"{os.path.basename(p)[:-5]:24s} {r['value']:9.1f} Mrays/s {r['ms_per_step']:9.1f} ms/step "
          f"{f['kernel']} frac={f['frac']} {st}")
