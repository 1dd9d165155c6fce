#!/usr/bin/env python3
"""Summarise the LUMO_SHADOW_STATS lines a diagnostics build (make variant NAME=sstats
DEVFLAGS=-DLUMO_SHADOW_STATS=1) prints to stderr: per record class (L / B record x environment
light x outcome) the count, mean traversal cost (AABB + kd + triangle steps), share of all cost
and the cost histogram (log2 bins); and the pair loop's lane efficiency."""
import sys

import numpy as np

tot = None
for line in open(sys.argv[1]):
    if line.startswith("LUMO_SHADOW_STATS"):
        v = np.array([int(x) for x in line.split()[1:]], dtype=np.float64)
        tot = v if tot is None else tot + v
if tot is None:
    sys.exit("no LUMO_SHADOW_STATS lines")
cls = tot[:216].reshape(12, 18)
all_cost = cls[:, 1].sum()
print(f"{'class':<22}{'count':>14}{'share':>8}{'mean cost':>11}{'cost share':>12}  histogram (log2 bins 0..15)")
for k in range(12):
    rec, env, out = k // 6, (k // 3) % 2, k % 3
    n, c = cls[k, 0], cls[k, 1]
    if n == 0:
        continue
    name = f"{'LB'[rec]} {'env' if env else 'lamp'} {['miss', 'occluded', 'visible'][out]}"
    hist = " ".join(f"{int(x)}" for x in cls[k, 2:])
    print(f"{name:<22}{int(n):>14}{n / cls[:, 0].sum():>8.3f}{c / n:>11.1f}{c / all_cost:>12.3f}  {hist}")
print(f"lane efficiency of the pair loop: {tot[216] / max(tot[217], 1):.3f}")
