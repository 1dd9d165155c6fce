"""Per-pass timeline of a rocprofv3 kernel trace (tools/profile.sh output): kernel time, gaps
between dispatches, and the share of the pass spent in bounces whose closest-hit kernel ran
below a duration threshold (the latency-bound tail).
Usage: python tools/timeline.py <run_kernel_trace.csv> [tail_us=60] [pass_index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tail_us = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
show = int(sys.argv[3]) if len(sys.argv) > 3 else -1
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
passes, cur = [], []
for r in rows:
    if "k_camera" in r["Kernel_Name"] and cur:
        passes.append(cur)
        cur = []
    cur.append(r)
passes.append(cur)
passes = [p for p in passes if any("k_camera" in r["Kernel_Name"] for r in p)]
tot = {"span": 0.0, "busy": 0.0, "tail_span": 0.0, "bounces": 0, "tail_bounces": 0}
for pi, p in enumerate(passes):
    s0 = int(p[0]["Start_Timestamp"])
    e1 = max(int(r["End_Timestamp"]) for r in p)
    tot["span"] += (e1 - s0) / 1e3
    tot["busy"] += sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in p) / 1e3
    # bounces: from k_bounce_begin to the next one
    idx = [i for i, r in enumerate(p) if "k_bounce_begin" in r["Kernel_Name"]]
    for a, b in zip(idx, idx[1:] + [len(p)]):
        seg = p[a:b]
        cl = [r for r in seg if "k_closest" in r["Kernel_Name"]]
        if not cl:
            continue
        tot["bounces"] += 1
        d = (int(cl[0]["End_Timestamp"]) - int(cl[0]["Start_Timestamp"])) / 1e3
        if d < tail_us:
            tot["tail_bounces"] += 1
            end = int(p[b]["Start_Timestamp"]) if b < len(p) else int(seg[-1]["End_Timestamp"])
            tot["tail_span"] += (end - int(seg[0]["Start_Timestamp"])) / 1e3
    if pi == show:
        prev = None
        for r in p:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"{r['Kernel_Name'][:44]:44s} {(e - s) / 1e3:9.1f} us  gap {((s - prev) / 1e3 if prev else 0):6.1f}")
            prev = e
n = len(passes)
print(f"passes {n}: span/pass {tot['span'] / n:.1f} us, kernel busy {tot['busy'] / tot['span']:.3f}, "
      f"bounces/pass {tot['bounces'] / n:.2f}, tail bounces/pass {tot['tail_bounces'] / n:.2f} "
      f"taking {tot['tail_span'] / tot['span']:.3f} of the span (closest < {tail_us} us)")
