"""Per-kernel sums of the counters tools/pmc_cmp.sh collected, one row per variant x kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict

KERNELS = ("k_camera", "k_closest_q", "k_closest", "k_shade_q", "k_shade", "k_shadow_q", "k_shadow", "k_nee_fold",
           "k_finish_film", "k_finish", "k_film", "k_ring", "k_bdpt_step", "k_bdpt_trace_a", "k_bdpt_vis")


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return name[:40]

root, names = sys.argv[1], [a for a in sys.argv[2:] if a != "--all"]
ALL = "--all" in sys.argv
for v in names:
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for p in glob.glob(os.path.join(root, v, "*", "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                k = short(r.get("Kernel_Name", ""))
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r.get("Dispatch_Id", ""))
    for k in sorted(acc, key=lambda k: -acc[k].get("SQ_WAVE_CYCLES", 0))[:6]:
        c = acc[k]
        if ALL:
            print(v, k, " ".join(f"{n}={x:.4g}" for n, x in sorted(c.items())))
            continue
        hit = c.get("TCC_HIT_sum", 0)
        miss = c.get("TCC_MISS_sum", 0)
        print(f"{v:6s} {k:14s} waves={c.get('SQ_WAVES', 0):.3g} valu={c.get('SQ_INSTS_VALU', 0):.4g} "
              f"salu={c.get('SQ_INSTS_SALU', 0):.4g} vmrd={c.get('SQ_INSTS_VMEM_RD', 0):.4g} "
              f"vmwr={c.get('SQ_INSTS_VMEM_WR', 0):.4g} wcyc={c.get('SQ_WAVE_CYCLES', 0):.4g} "
              f"wait={c.get('SQ_WAIT_ANY', 0):.4g} act={c.get('SQ_ACTIVE_INST_ANY', 0):.4g} "
              f"l2hit={hit / max(hit + miss, 1):.3f} l2req={hit + miss:.4g} tcp={c.get('TCP_TOTAL_CACHE_ACCESSES_sum', 0):.4g}")
