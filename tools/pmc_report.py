"""Per-kernel sums of the counters collected by tools/pmc.sh (all tags given)."""
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float))
for tag in sys.argv[1:]:
    for p in glob.glob(f"gpurun_out/pmc/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            n = r["Kernel_Name"]
            k = next((x for x in ("k_closest", "k_shade", "k_shadow", "k_camera", "k_resolve", "k_film", "k_finish", "k_ring") if x in n), None)
            if k:
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:.4g}")
    if "SQ_THREAD_CYCLES_VALU" in d and "SQ_ACTIVE_INST_VALU" in d and d["SQ_ACTIVE_INST_VALU"]:
        print("   => VALU lane utilization (thread cycles / (active inst cycles x 64)):",
              round(d["SQ_THREAD_CYCLES_VALU"] / (d["SQ_ACTIVE_INST_VALU"] * 64), 3))
    if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d and d["SQ_WAVES"]:
        print("   => VALU insts per wave:", round(d["SQ_INSTS_VALU"] / d["SQ_WAVES"]))
