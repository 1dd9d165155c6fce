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
    for k in ("k_camera", "k_closest", "k_shade", "k_shadow_queue", "k_shadow", "k_resolve", "k_finish_film",
              "k_finish", "k_film", "k_ring", "k_init_mj", "k_init_seeds", "k_trace", "k_bdpt_redo", "k_bdpt_taps",
              "k_bdpt_trace_a", "k_bdpt_vis", "k_bdpt_eval_a", "k_bdpt_paths", "k_bdpt_step", "k_bdpt_tail",
              "k_bdpt_fold", "k_bdpt", "k_nee_gen", "k_nee_fold", "k_calib_read8", "k_calib_write8",
              "k_bounce_begin", "k_task_tap_ranges"):
        if k in name:
            return k
    return name[:60]


UNITS = {"k_bounce_q+k_bounce_tail": ("k_bounce_q", "k_bounce_tail"),
         "k_bdpt_trace_a+k_bdpt_vis": ("k_bdpt_trace_a", "k_bdpt_vis")}


def union_ns(iv):
    """Length of the union of [start, end] intervals: the time at least one launch ran."""
    total, lo, hi = 0, None, None
    for a, b in sorted(iv):
        if hi is not None and a <= hi:
            hi = max(hi, b)
            continue
        if hi is not None:
            total += hi - lo
        lo, hi = a, b
    return total + (hi - lo if hi is not None else 0)


res = defaultdict(lambda: {"launches": 0, "total_ns": 0})
ivs = defaultdict(list)
for r in rows("trace/**/*kernel_trace.csv"):
    k = short(r.get("Kernel_Name", ""))
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    res[k]["launches"] += 1
    res[k]["total_ns"] += b - a
    ivs[k].append((a, b))
    # resources of the code object (the kernel trace carries them per dispatch): registers,
    # scratch bytes per lane, LDS per workgroup; the register-limited waves per SIMD follow
    # (512 VGPRs per SIMD lane, arch + accumulation registers in granules of 8).  On gfx950 the
    # trace's VGPR_Count is half the allocation the compiler reports (NumVgprs: 168 for the C1 fused
    # kernel, traced as 84; 256 for the tail kernel, traced as 128), so it is doubled here.
    if "VGPR_Count" in r:
        vg = 2 * int(r["VGPR_Count"]) + int(r.get("Accum_VGPR_Count") or 0)
        wg = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 0)
        res[k]["resources"] = {"vgpr": vg, "sgpr": int(r.get("SGPR_Count") or 0),
                               "scratch_bytes_per_lane": int(r.get("Scratch_Size") or 0),
                               "lds_bytes_per_workgroup": int(r.get("LDS_Block_Size") or 0), "workgroup": wg,
                               "waves_per_simd_by_vgpr": min(8, 512 // max(8, (vg + 7) // 8 * 8))}
for k, v in res.items():
    v["avg_us"] = v["total_ns"] / max(v["launches"], 1) / 1e3
    v["busy_ms"] = union_ns(ivs[k]) / 1e6  # overlapping launches (several streams) counted once
for u, parts in UNITS.items():
    if all(p in res for p in parts):
        iv = [x for p in parts for x in ivs[p]]
        n = sum(res[p]["launches"] for p in parts)
        tot = sum(res[p]["total_ns"] for p in parts)
        res[u] = {"launches": n, "total_ns": tot, "avg_us": tot / n / 1e3, "busy_ms": union_ns(iv) / 1e6}
if ivs:
    allv = [x for v in ivs.values() for x in v]
    res["_gpu"] = {"busy_ms": union_ns(allv) / 1e6, "span_ms": (max(b for _, b in allv) - min(a for a, _ in allv)) / 1e6}
# SQ pass (tools/profile.sh "valu"): VALU lane activity, wave cycles and waits, per launch
SQ = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
      "SQ_INSTS_FLAT", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR")
sq = defaultdict(lambda: defaultdict(lambda: [0.0, set()]))
for r in rows("valu/**/*counter_collection.csv"):
    c = r.get("Counter_Name")
    if c in SQ:
        k = short(r.get("Kernel_Name", ""))
        sq[k][c][0] += float(r["Counter_Value"])
        sq[k][c][1].add(r.get("Dispatch_Id"))
for k, d in sq.items():
    n = max(len(d["SQ_INSTS_VALU"][1]), 1)
    per = {c: d[c][0] / max(len(d[c][1]), 1) for c in d}
    res[k]["sq_per_launch"] = per
    if per.get("SQ_ACTIVE_INST_VALU"):
        lanes = per["SQ_THREAD_CYCLES_VALU"] / per["SQ_ACTIVE_INST_VALU"]
        res[k]["lanes_active_per_valu_inst"] = lanes
        res[k]["valu_lane_ops_per_launch"] = per["SQ_INSTS_VALU"] * lanes
    if per.get("SQ_WAVE_CYCLES"):
        res[k]["wait_any_frac"] = per["SQ_WAIT_ANY"] / per["SQ_WAVE_CYCLES"]
for u, parts in UNITS.items():
    if all(p in res and "valu_lane_ops_per_launch" in res[p] for p in parts):
        n = sum(res[p]["launches"] for p in parts)
        ops = sum(res[p]["valu_lane_ops_per_launch"] * res[p]["launches"] for p in parts) / n
        ins = sum(res[p]["sq_per_launch"]["SQ_INSTS_VALU"] * res[p]["launches"] for p in parts) / n
        res[u]["valu_lane_ops_per_launch"] = ops
        res[u]["lanes_active_per_valu_inst"] = ops / ins
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
