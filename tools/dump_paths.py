"""Dump GPU and oracle per-path records of one task to gpurun_out/ (diagnostics)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import lumo_amd as L
import oracle_ffi as O
from parity import gpu_paths

w, h, spp, tile = (int(x) for x in sys.argv[1:5])
sc = L.Scene.cornell_box(); cam = L.Camera.cornell_box((w, h))
dev = L.Device(0); dev.upload(sc, cam)
task = L.make_tasks(w, h, spp, 0x5EED1234)[tile]
g = gpu_paths(dev, task); o = O.trace_paths(sc.desc(), cam.desc, task)
np.savez(os.path.join(ROOT, "gpurun_out", f"paths_{w}x{h}_{spp}_{tile}.npz"),
         **{"g_" + k: v for k, v in g.items()}, **{"o_" + k: v for k, v in o.items()})
bad = np.nonzero(g["depth"] != o["depth"])[0]
print("mismatch", len(bad), "of", len(g["depth"]), bad[:20])
