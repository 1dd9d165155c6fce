"""Offline A/B of the wide BVH's build parameters (wbvh_build.h WBVH_LEAF_MAX / WBVH_C_TRAV): builds
oracle variants with the macros set and reports the wide walks' counters per query on a few tiles
of a benchmark scene rendered by the oracle (wavefront order, the real ray mix).
    python tools/wbvh_params.py <c1|c2|c3|c4> "<leaf>:<ctrav>" ..."""
import ctypes as C
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ffi as O  # noqa: E402
import lumo_amd as L  # noqa: E402
from lumo_amd import scenes  # noqa: E402


def variant(leaf, ctrav):
    out = f"/tmp/oracle_wbvh_{leaf}_{ctrav}.so"
    if not os.path.exists(out):
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-shared",
                        f"-DWBVH_LEAF_MAX={leaf}", f"-DWBVH_C_TRAV={ctrav}", "-o", out,
                        os.path.join(ROOT, "oracle/src/oracle.cpp"), "-lpthread"], check=True)
    return out


def main():
    cfg = sys.argv[1]
    if cfg == "c2":
        sc, cam = scenes.dragon(), scenes.default_camera((1920, 1080))
    elif cfg == "c3":
        sc, cam = scenes.bistro(), scenes.bistro_camera((1920, 1080))
    elif cfg == "c4":
        sc, cam = scenes.caustics(), scenes.caustics_camera((1024, 1024))
    else:
        sc, cam = L.Scene.cornell_box(), L.Camera.cornell_box((1024, 1024))
    sc.build()
    W, H = int(cam.desc.width), int(cam.desc.height)
    tasks = L.make_tasks(W, H, 4, 0x5EED1234)
    sub = tasks[:: max(1, len(tasks) // 48)][:48]
    integ = L.Integrator.BDPathTrace if cfg == "c4" else 0
    for spec in sys.argv[2:]:
        leaf, ctrav = spec.split(":")
        path = variant(leaf, ctrav)
        t0 = time.time()
        _, res, c = O.render_tasks(sc.desc(), cam.desc, sub, O.WAVEFRONT, 8, path=path, accel=1, integrator=integ,
                                   splats_out=[] if integ else None)
        q = c.closest_queries + c.shadow_queries
        lib = O.load(path)
        info = (C.c_int64 * 8)()
        lib.oracle_wide_export(C.byref(sc.desc()), info, None, None, None, None)
        print(f"leaf {leaf} ctrav {ctrav}: nodes/q {c.kd_nodes / q:.2f} boxes/q {c.aabb_tests / q:.2f} "
              f"tris/q {c.tri_tests / q:.2f}  cost(3:1) {(3 * c.kd_nodes + c.tri_tests) / q:.2f}  "
              f"[{int(info[1])} nodes, stack {int(info[3])}, depth {int(info[4])}] {time.time() - t0:.1f} s",
              flush=True)


if __name__ == "__main__":
    main()
