import json, sys
for v in sys.argv[1:]:
    d = json.load(open(f"gpurun_out/ab_{v}.json")); r = d["roofline"]
    print(f"{v:8s} {d['value']:9.1f} Mrays/s {d['ms_per_step']:9.1f} ms/step  {r['kernel']} frac={r['frac']}  " +
          " ".join(f"{k}={v['ms']:.0f}" for k, v in r["stages"].items()))
