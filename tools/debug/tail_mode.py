"""Debug: tail-kernel-only bounce mode (fused 0, tail 2^30, pipeline 0) on Cornell 48x40 @ 24:
which tiles differ from the oracle, whether repeated renders agree, and per-path diffs."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import lumo_amd as L
import oracle_ffi as O
from lumo_amd import _ffi
from parity import gpu_paths
lib = _ffi.load()
mode = [int(x) for x in sys.argv[1:4]] if len(sys.argv) > 3 else [0, 1 << 30, 0]
lib.lumo_set_bounce_mode(*mode)
sc = L.Scene.cornell_box()
cam = L.Camera.cornell_box((48, 40))
d = L.Device(0)
d.upload(sc, cam)
tasks = L.make_tasks(48, 40, 24, 0x5EED1234)
a, ra = d.render_tasks(tasks)
b, rb = d.render_tasks(tasks)
o, ro, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
print("mode", mode, "repeat equal:", all(np.array_equal(x, y) for x, y in zip(a, b)))
bad = [i for i, (x, y) in enumerate(zip(a, o)) if not np.array_equal(x, y)]
print("bad tiles", bad, "of", len(tasks))
print("rays", [(r.num_rays, q.num_rays, r.num_queries, q.num_queries) for r, q in zip(ra, ro)][:4])
for i in bad[:3]:
    g = gpu_paths(d, tasks[i])
    p = O.trace_paths(sc.desc(), cam.desc, tasks[i])
    for k in ("depth", "raster", "lam", "radiance"):
        diff = np.nonzero(np.any(np.atleast_2d(g[k].T).T != np.atleast_2d(p[k].T).T, axis=-1) if g[k].ndim > 1 else g[k] != p[k])[0]
        print(" task", i, k, "paths differing:", len(diff), diff[:10])
d.close()
