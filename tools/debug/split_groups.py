"""Debug: render the mid-size Bistro stand-in (n_shadow > 1, split schedule) with LUMO_SPLIT_PIPE /
LUMO_SPLIT_GROUPS from argv and list the tiles that differ from the sequential schedule and from
the oracle.  Usage: python tools/debug/split_groups.py K G"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import lumo_amd as L
import oracle_ffi as O
from lumo_amd import scenes
from lumo_amd.procedural import bistro_standin

K, G = sys.argv[1], sys.argv[2]
sc = scenes.bistro(bistro_standin(groups=48, lamps=160, n=8)).build()
cam = scenes.bistro_camera((64, 48))
tasks = L.make_tasks(64, 48, 9, 0x5EED1234)


def render(k, g):
    os.environ["LUMO_SPLIT_PIPE"], os.environ["LUMO_SPLIT_GROUPS"] = str(k), str(g)
    d = L.Device(0)
    d.upload(sc, cam)
    b, r = d.render_tasks(tasks)
    d.close()
    return b, r


seq, _ = render(1, 1)
par, _ = render(K, G)
ob, _, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
print("tasks", len(tasks), "first px", [tuple(t.px_min) for t in tasks[:4]])
print("seq vs oracle bad:", [i for i, (a, b) in enumerate(zip(seq, ob)) if not np.array_equal(a, b)])
print(f"K={K} G={G} vs oracle bad:", [i for i, (a, b) in enumerate(zip(par, ob)) if not np.array_equal(a, b)])
print(f"K={K} G={G} vs seq bad:", [i for i, (a, b) in enumerate(zip(par, seq)) if not np.array_equal(a, b)])
