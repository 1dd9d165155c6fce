"""Offline estimate (CPU, no product code): would C3's shadow rays walk fewer wide nodes if their
any-hit walk first searched a subtree around the ray's origin?

Shadow rays are built like the path tracer's light-sampled NEE records: camera rays of the C3
camera hit the scene (oracle, wide accel, with the hit triangle), and each hit sends a ray to a
uniform point of a uniform lamp triangle.  For every ray this walks the exported wide BVH
(tests/oracle_ffi.wide_export) in Python:
* plain: the objects' tree from the root, any hit, children that pass in node order;
* hint K: first the subtree of the origin leaf's K-th ancestor; if it holds no occluder, the plain
  walk (the subtree's nodes are counted twice then).
Nodes visited per ray are reported, and for an 8-wide tree made by opening each node's
largest interior children (up to 8 entries) the nodes and child boxes per ray.  Triangle tests use Moller-Trumbore in f64 (an estimate, not
lumo's watertight test).  Usage: python tools/hint_estimate.py [n_rays]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import lumo_amd as L  # noqa: E402
import oracle_ffi as O  # noqa: E402
from lumo_amd import scenes  # noqa: E402

NONE = -(1 << 31)


def main():
    n_rays = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    rng = np.random.default_rng(5)
    sc = scenes.bistro().build()
    d = sc.desc()
    acc = O.wide_export(d)
    nodes, tv = acc["nodes"], acc["tv"]
    lo = np.stack([nodes["lo"][:, a, :] for a in range(3)], 1).astype(np.float64)  # [node, axis, child]
    hi = np.stack([nodes["hi"][:, a, :] for a in range(3)], 1).astype(np.float64)
    ref, cnt = nodes["ref"], nodes["n"]
    # parents and the leaf (node) of every triangle record of the objects' tree
    parent = np.full(len(nodes), -1, dtype=np.int64)
    rec_node = {}
    stack = [acc["obj_root"]]
    while stack:
        i = stack.pop()
        for k in range(cnt[i]):
            r = int(ref[i, k])
            if r >= 0:
                parent[r] = i
                stack.append(r)
            else:
                x = ~r
                for j in range((x >> 4), (x >> 4) + (x & 15)):
                    rec_node[int(acc["tri"][j])] = i
    # shadow ray origins: closest hits of camera-like rays
    cam_o = np.array([-16.0, 5.0, -1.0])
    dirs = rng.normal(size=(4 * n_rays, 3)) * 0.35 + (np.zeros(3) - cam_o) / np.linalg.norm(cam_o)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    o = np.repeat(cam_o[None], len(dirs), 0)
    t, kind, obj, prim, _ = O.trace(d, o, dirs, accel=1, with_prim=True)
    ok = (kind == 1) & np.isfinite(t) & np.isin(prim, list(rec_node.keys()))
    o, dirs, t, prim = o[ok][:n_rays], dirs[ok][:n_rays], t[ok][:n_rays], prim[ok][:n_rays]
    p = o + dirs * t[:, None]
    v = np.ctypeslib.as_array(d.vertices, shape=(d.num_vertices, 3))
    tris = np.ctypeslib.as_array(d.triangles, shape=(d.num_triangles,))
    lights = np.ctypeslib.as_array(d.lights, shape=(d.num_lights,))
    lamp_tris = np.concatenate([np.arange(lt["tri_base"], lt["tri_base"] + max(lt["num_tris"], 1))
                                for lt in lights if lt["type"] != 3])
    pick = lamp_tris[rng.integers(0, len(lamp_tris), size=len(p))]
    a, b, c = (v[tris["v"][pick][:, k]] for k in range(3))
    uu = rng.uniform(size=(len(p), 2))
    s = np.sqrt(uu[:, :1])
    q = (1 - s) * a + s * (1 - uu[:, 1:]) * b + s * uu[:, 1:] * c
    # origin offset off the surface along the ray back (an estimate of ray_origin)
    sd = q - p
    dist = np.linalg.norm(sd, axis=1)
    sd /= dist[:, None]
    origin = p - dirs * 1e-4 * np.maximum(1.0, t)[:, None]
    # only rays a Lambertian surface would trace: the lamp on the viewer's side of the surface (a
    # light behind it has BSDF pdf 0 and is answered without a walk, LUMO_SKIP_DEAD)
    ta, tb, tc = (v[tris["v"][prim][:, k]] for k in range(3))
    ng = np.cross(tb - ta, tc - ta)
    keep = np.sign(np.sum(ng * sd, 1)) == np.sign(np.sum(ng * -dirs, 1))
    origin, sd, dist, prim = origin[keep], sd[keep], dist[keep], prim[keep]

    def tri_hit(j, ro, rd, tmax):
        A, B, C = tv[j, 0:3], tv[j, 3:6], tv[j, 6:9]
        e1, e2 = B - A, C - A
        h = np.cross(rd, e2)
        det = e1 @ h
        if abs(det) < 1e-14:
            return False
        f = 1.0 / det
        sv = ro - A
        u = f * (sv @ h)
        if u < 0 or u > 1:
            return False
        qv = np.cross(sv, e1)
        w = f * (rd @ qv)
        if w < 0 or u + w > 1:
            return False
        tt = f * (e2 @ qv)
        return 1e-6 < tt < tmax

    def walk(root, ro, rd, tmax):
        inv = 1.0 / np.where(rd == 0, 1e-300, rd)
        st, nv = [root], 0
        while st:
            i = st.pop()
            nv += 1
            t0 = (lo[i] - ro[:, None]) * inv[:, None]
            t1 = (hi[i] - ro[:, None]) * inv[:, None]
            tn = np.minimum(t0, t1).max(0)
            tf = np.maximum(t0, t1).min(0)
            hit = (tn <= tf) & (tf >= 0) & (tn <= tmax)
            for k in range(cnt[i] - 1, -1, -1):
                if not hit[k]:
                    continue
                r = int(ref[i, k])
                if r >= 0:
                    st.append(r)
                else:
                    x = ~r
                    for j in range((x >> 4), (x >> 4) + (x & 15)):
                        if tri_hit(j, ro, rd, tmax):
                            return True, nv
        return False, nv

    # 8-wide estimate: each 8-wide node = a 4-wide node with its largest-area interior children
    # opened until 8 entries; walk counts 8-wide nodes and child boxes tested
    def area(i, k):
        e = hi[i, :, k] - lo[i, :, k]
        return e[0] * e[1] + e[1] * e[2] + e[2] * e[0]
    wide8 = {}

    def entries8(i):
        if i in wide8:
            return wide8[i]
        ent = [(i, k) for k in range(cnt[i])]
        while True:
            inner = [e for e in ent if int(ref[e[0], e[1]]) >= 0]
            if not inner:
                break
            e = max(inner, key=lambda e: area(*e))
            c = int(ref[e[0], e[1]])
            if len(ent) - 1 + cnt[c] > 8:
                break
            ent.remove(e)
            ent += [(c, k) for k in range(cnt[c])]
        wide8[i] = ent
        return ent

    def walk8(root, ro, rd, tmax):
        inv = 1.0 / np.where(rd == 0, 1e-300, rd)
        st, nv, nb = [root], 0, 0
        while st:
            i = st.pop()
            nv += 1
            ent = entries8(i)
            nb += len(ent)
            for (nd, k) in reversed(ent):
                t0 = (lo[nd, :, k] - ro) * inv
                t1 = (hi[nd, :, k] - ro) * inv
                tn, tf = np.minimum(t0, t1).max(), np.maximum(t0, t1).min()
                if not (tn <= tf and tf >= 0 and tn <= tmax):
                    continue
                r = int(ref[nd, k])
                if r >= 0:
                    st.append(r)
                else:
                    x = ~r
                    for j in range((x >> 4), (x >> 4) + (x & 15)):
                        if tri_hit(j, ro, rd, tmax):
                            return True, nv, nb
        return False, nv, nb

    n8, b8 = [], []
    for r in range(min(len(origin), 600)):
        _, nv, nb = walk8(acc["obj_root"], origin[r], sd[r], dist[r] * (1 - 1e-6))
        n8.append(nv)
        b8.append(nb)

    K = (1, 2, 3)
    plain, hint = [], {k: [] for k in K}
    found = {k: 0 for k in K}
    occl = 0
    for r in range(len(origin)):
        ro, rd, tmax = origin[r], sd[r], dist[r] * (1 - 1e-6)
        occ, nv = walk(acc["obj_root"], ro, rd, tmax)
        occl += occ
        plain.append(nv)
        for k in K:
            a_ = rec_node[int(prim[r])]
            for _ in range(k):
                a_ = parent[a_] if parent[a_] >= 0 else a_
            h, n1 = walk(a_, ro, rd, tmax)
            found[k] += h
            hint[k].append(n1 if h else n1 + nv)
    n = len(plain)
    print(f"rays {n}, occluded {occl / n:.3f}, plain nodes per ray {np.mean(plain):.2f}")
    print(f"8-wide (first {len(n8)} rays): nodes per ray {np.mean(n8):.2f} against {np.mean(plain[:len(n8)]):.2f}, "
          f"child boxes per ray {np.mean(b8):.1f}")
    for k in K:
        print(f"hint K={k}: nodes per ray {np.mean(hint[k]):.2f} ({np.mean(hint[k]) / np.mean(plain) - 1:+.1%}), "
              f"occluder found in the subtree for {found[k] / max(occl, 1):.3f} of the occluded rays")


if __name__ == "__main__":
    main()
