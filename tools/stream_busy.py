"""Occupancy of the last rendered frame in a rocprofv3 kernel trace: the frame's span, the union of
all its kernels' intervals (GPU busy), the average number of kernels running at once, and per
kernel family and per hardware queue the launch count, summed duration and busy union.  The frame
is the render call that starts at the last k_init_seeds dispatch (one per lumo_render_tiles chunk).
Usage: python tools/stream_busy.py <kernel_trace.csv>"""
import csv
import json
import re
import sys


def union(iv):
    iv = sorted(iv)
    tot, lo, hi = 0, None, None
    for a, b in iv:
        if hi is not None and a <= hi:
            hi = max(hi, b)
            continue
        if hi is not None:
            tot += hi - lo
        lo, hi = a, b
    if hi is not None:
        tot += hi - lo
    return tot


def family(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n).replace("void ", "").split("::")[-1].strip()
    if "k_bounce_q" in name:
        n += "<TAIL>" if re.search(r"k_bounce_q<[^>]*true>", name) else "<head>"
    return n


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    for r in rows:
        r["a"], r["b"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    starts = [r["a"] for r in rows if "k_init_seeds" in r["Kernel_Name"]]
    t0 = max(starts)
    fr = [r for r in rows if r["a"] >= t0]
    t1 = max(r["b"] for r in fr)
    span = t1 - t0
    busy = union([(r["a"], r["b"]) for r in fr])
    out = {"span_ms": span / 1e6, "busy_ms": busy / 1e6, "busy_frac": busy / span,
           "avg_running": sum(r["b"] - r["a"] for r in fr) / span, "families": {}, "queues": {}}
    fams = {}
    for r in fr:
        fams.setdefault(family(r["Kernel_Name"]), []).append((r["a"], r["b"]))
    for k, iv in sorted(fams.items(), key=lambda kv: -sum(b - a for a, b in kv[1])):
        out["families"][k] = {"n": len(iv), "sum_ms": sum(b - a for a, b in iv) / 1e6, "busy_ms": union(iv) / 1e6,
                              "avg_us": sum(b - a for a, b in iv) / len(iv) / 1e3}
    qk = "Queue_Id" if "Queue_Id" in fr[0] else ("Stream_Id" if "Stream_Id" in fr[0] else None)
    if qk:
        qs = {}
        for r in fr:
            qs.setdefault(r[qk], []).append((r["a"], r["b"]))
        for k, iv in qs.items():
            out["queues"][k] = {"n": len(iv), "sum_ms": sum(b - a for a, b in iv) / 1e6, "busy_ms": union(iv) / 1e6}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
