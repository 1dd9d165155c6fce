"""Bounce-by-bounce trace of one path on GPU and in the oracle (diagnostics)."""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import lumo_amd as L
from lumo_amd import _ffi
import oracle_ffi as O

w, h, spp, tile = (int(x) for x in sys.argv[1:5])
pairs = [tuple(int(y) for y in x.split(":")) for x in sys.argv[5:]]
sc = L.Scene.cornell_box(); cam = L.Camera.cornell_box((w, h))
dev = L.Device(0); dev.upload(sc, cam)
task = L.make_tasks(w, h, spp, 0x5EED1234)[tile]
lib = _ffi.load(); olib = O.load()
lib.lumo_debug_trace.argtypes = [C.c_void_p, C.POINTER(_ffi.TileTask), C.c_int, C.c_int, _ffi.c_double_p, C.POINTER(C.c_int)]
olib.oracle_debug_trace.argtypes = [C.POINTER(_ffi.SceneDesc), C.POINTER(_ffi.CameraDesc), C.POINTER(_ffi.TileTask), C.c_int, C.c_int, _ffi.c_double_p, C.POINTER(C.c_int)]
np.set_printoptions(precision=17, linewidth=250)
for (ps, px) in pairs:
    g = np.zeros((64, 20)); o = np.zeros((64, 20)); ng = C.c_int(); no = C.c_int()
    assert lib.lumo_debug_trace(dev.ctx, C.byref(task), ps, px, g.ctypes.data_as(_ffi.c_double_p), C.byref(ng)) == 0
    d = sc.desc()
    assert olib.oracle_debug_trace(C.byref(d), C.byref(cam.desc), C.byref(task), ps, px, o.ctypes.data_as(_ffi.c_double_p), C.byref(no)) == 0
    print(f"=== pass {ps} pixel {px}: gpu bounces {ng.value} oracle {no.value}")
    for i in range(max(ng.value, no.value)):
        print("G", i, g[i].tolist()); print("O", i, o[i].tolist())
        diff = np.nonzero(g[i] != o[i])[0]
        print("  differs at", diff.tolist())
