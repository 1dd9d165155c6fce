"""oracle(wide) against oracle(lumo) on the same rays: closest hits (t, kind, object)
and light visibility, with the mismatches classified.  Usage:
    python tools/wide_vs_lumo.py <scene: cornell|dragon|bistro|caustics|zoo> [n_rays] [seed]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_ffi as O  # noqa: E402
from lumo_amd import scenes  # noqa: E402
from test_gpu_scale import _closest_rays, _visibility_rays  # noqa: E402


def build(name):
    if name == "cornell":
        return scenes.cornell().build(), (278.0, 273.0, -800.0)
    if name == "dragon":
        return scenes.dragon().build(), (0.0, 0.0, 0.0)
    if name == "bistro":
        return scenes.bistro().build(), (-16.0, 5.0, -1.0)
    if name == "caustics":
        return scenes.caustics().build(), (0.0, 0.0, 2.0)
    import scenes as T
    return T.material_zoo().build(), (0.0, 0.0, 0.0)


def compare(sc, o, d, lights=None):
    t0 = time.time()
    a = O.trace(sc.desc(), o, d, lights)
    t1 = time.time()
    b = O.trace(sc.desc(), o, d, lights, accel=1)
    t2 = time.time()
    same_t = (a[0] == b[0]) | (np.isinf(a[0]) & np.isinf(b[0]))
    same = same_t & (a[1] == b[1]) & (a[2] == b[2])
    n = len(o)
    out = dict(n=n, t_equal=int(same_t.sum()), all_equal=int(same.sum()),
               t_only_kind_obj_differ=int((same_t & ~same).sum()),
               lumo_s=round(t1 - t0, 2), wide_s=round(t2 - t1, 2),
               lumo_cnt=[a[3].aabb_tests / n, a[3].kd_nodes / n, a[3].tri_tests / n],
               wide_cnt=[b[3].aabb_tests / n, b[3].kd_nodes / n, b[3].tri_tests / n])
    bad = np.nonzero(~same_t)[0]
    out["t_differ"] = len(bad)
    # classes: lumo misses what the wide walk hits; the wide walk misses what lumo hits; both hit
    # with different t (near-coincident surfaces: a light on the ceiling, a tie in another order)
    am, bm = np.isinf(a[0][bad]), np.isinf(b[0][bad])
    out["lumo_miss_wide_hit"] = int((am & ~bm).sum())
    out["wide_miss_lumo_hit"] = int((~am & bm).sum())
    both = ~am & ~bm
    out["both_hit_t_differ"] = int(both.sum())
    if both.any():
        r = np.abs(a[0][bad][both] - b[0][bad][both]) / np.abs(a[0][bad][both])
        out["both_hit_rel_t_max"] = float(r.max())
        out["both_hit_wide_closer"] = int((b[0][bad][both] < a[0][bad][both]).sum())
    if len(bad):
        out["t_differ_examples"] = [(int(i), float(a[0][i]), float(b[0][i]), int(a[1][i]), int(b[1][i]),
                                     int(a[2][i]), int(b[2][i])) for i in bad[:5]]
    return out


if __name__ == "__main__":
    name = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 16
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 11
    t = time.time()
    sc, eye = build(name)
    print("build", round(time.time() - t, 1), "s", flush=True)
    o, d = _closest_rays(sc.desc(), eye, n, seed)
    print("closest", compare(sc, o, d), flush=True)
    o, d, li = _visibility_rays(sc.desc(), n, seed + 1)
    print("visibility", compare(sc, o, d, li), flush=True)
