"""Summarise rocprofv3 CSV output of tools/profile.sh: per-kernel launches, average duration
(kernel trace) and HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE passes.
gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of wide
coalesced reads -> reported both raw and x2; WRITE_SIZE is taken as is. Units: KB -> bytes."""
import csv, glob, json, os, sys
from collections import defaultdict

out = sys.argv[1]


def rows(pattern):
    for p in glob.glob(os.path.join(out, pattern), recursive=True):
        with open(p) as f:
            yield from csv.DictReader(f)


def short(name):
    if "k_bounce_q" in name:  # k_bounce_q<STK, LDS, FX, TAIL>: the fused bounce and the tail kernel
        return "k_bounce_tail" if name.split("(")[0].rstrip().endswith("true>") else "k_bounce_q"
    for k in ("k_camera", "k_closest", "k_shade", "k_shadow_queue", "k_shadow", "k_resolve", "k_finish_film", "k_finish", "k_film",
              "k_ring", "k_init_mj", "k_init_seeds", "k_trace", "k_bdpt_redo", "k_bdpt_taps", "k_bdpt_trace_a",
              "k_bdpt_vis", "k_bdpt_eval_a", "k_bdpt_paths", "k_bdpt_step", "k_bdpt_fold", "k_bdpt", "k_nee_gen", "k_nee_fold",
              "k_calib_read8", "k_calib_write8",
              "k_bounce_begin", "k_task_tap_ranges"):
        if k in name:
            return k
    return name[:60]


res = defaultdict(lambda: {"launches": 0, "total_ns": 0})
for r in rows("trace/**/*kernel_trace.csv"):
    k = short(r.get("Kernel_Name", ""))
    res[k]["launches"] += 1
    res[k]["total_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, v in res.items():
    v["avg_us"] = v["total_ns"] / max(v["launches"], 1) / 1e3
for tag, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    acc = defaultdict(lambda: [0.0, 0])
    for r in rows(f"{tag}/**/*counter_collection.csv"):
        if r.get("Counter_Name") != ctr:
            continue
        k = short(r.get("Kernel_Name", ""))
        acc[k][0] += float(r["Counter_Value"]) * 1024.0
        acc[k][1] += 1
    for k, (b, n) in acc.items():
        res[k][ctr.lower() + "_bytes_per_launch"] = b / max(n, 1)
for k, v in res.items():
    if "fetch_size_bytes_per_launch" in v and "write_size_bytes_per_launch" in v:
        v["hbm_bytes_per_launch"] = 2 * v["fetch_size_bytes_per_launch"] + v["write_size_bytes_per_launch"]
        v["hbm_bytes_per_launch_raw"] = v["fetch_size_bytes_per_launch"] + v["write_size_bytes_per_launch"]
print(json.dumps(dict(res), indent=1, sort_keys=True))
