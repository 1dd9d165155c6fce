"""Copy a tools/profile.sh run into profiles/<round>/ and refresh profiles/pmc_traffic.json
(HBM bytes per launch per kernel, read by bench.py's roofline).
Usage: python tools/update_traffic.py gpurun_out/prof/<tag> <round> [workload=c1]"""
import json
import os
import shutil
import sys

src, rnd = sys.argv[1], sys.argv[2]
workload = sys.argv[3] if len(sys.argv) > 3 else "c1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(ROOT, "profiles", rnd, workload)
os.makedirs(dst, exist_ok=True)
summary = json.load(open(os.path.join(src, "summary.json")))
shutil.copy(os.path.join(src, "summary.json"), os.path.join(dst, "rocprof_summary.json"))
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
for name in ("bench_trace.json", "bench_fetch.json", "bench_write.json", "bench_valu.json"):
    p = os.path.join(src, name)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, name.replace("bench_", "bench_under_rocprof_")))
path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
try:
    table = json.load(open(path))
except (OSError, ValueError):
    table = {}
table["correction"] = ("hbm = 2*FETCH_SIZE + WRITE_SIZE (gfx950: FETCH_SIZE counts half of wide coalesced reads, "
                       "MI355X_MICROARCH.md HBM section); raw = FETCH_SIZE + WRITE_SIZE. Bytes per launch.")
out = {"source": f"profiles/{rnd}/{workload}/rocprof_summary.json (tools/profile.sh: separate FETCH_SIZE and "
                 "WRITE_SIZE passes, no traces)"}
KEYS = ("hbm_bytes_per_launch", "hbm_bytes_per_launch_raw", "avg_us", "launches", "busy_ms",
        "valu_lane_ops_per_launch", "lanes_active_per_valu_inst", "wait_any_frac")
for k, v in summary.items():
    if k.startswith("k_") and "hbm_bytes_per_launch" in v:
        out[k] = {kk: v[kk] for kk in KEYS if kk in v}
if "k_bdpt_trace_a" in out and "k_bdpt_vis" in out:  # bench.py's BDPT connection unit: both kernels
    # per bench.py launch: its stage timers count one trace launch (two k_bdpt_trace_a dispatches,
    # one per trace list) and one visibility launch per pass and task group.  k_bdpt_vis is skipped
    # in a pass without (b) items, so the pass count is the larger of the two estimates.
    a, b = out["k_bdpt_trace_a"], out["k_bdpt_vis"]
    n = 2 * max(b["launches"], (a["launches"] + 1) // 2)
    out["k_bdpt_trace_a+k_bdpt_vis"] = {
        kk: (a[kk] * a["launches"] + b[kk] * b["launches"]) / n
        for kk in ("hbm_bytes_per_launch", "hbm_bytes_per_launch_raw", "avg_us")}
    out["k_bdpt_trace_a+k_bdpt_vis"]["launches"] = n
for a_k, b_k in (("k_bounce_q", "k_bounce_tail"),):  # bench.py's fused unit: both kernels
    if a_k in out and b_k in out:
        a, b = out[a_k], out[b_k]
        n = a["launches"] + b["launches"]
        out[a_k + "+" + b_k] = {
            kk: (a[kk] * a["launches"] + b[kk] * b["launches"]) / n
            for kk in ("hbm_bytes_per_launch", "hbm_bytes_per_launch_raw", "avg_us")}
        out[a_k + "+" + b_k]["launches"] = n
for u in ("k_bounce_q+k_bounce_tail", "k_bdpt_trace_a+k_bdpt_vis"):  # union busy time, VALU of the unit
    if u in out and u in summary:
        out[u].update({kk: summary[u][kk] for kk in ("busy_ms", "valu_lane_ops_per_launch", "lanes_active_per_valu_inst")
                       if kk in summary[u]})
table[workload] = out
json.dump(table, open(path, "w"), indent=1, sort_keys=True)
print("updated", dst)
