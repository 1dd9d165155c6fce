"""The wide accel mode on the CPU: the structure the upload builds
(lumo_amd/csrc/common/wbvh_build.h, exported through the oracle) and how the oracle's wide walk
relates to its restatement of lumo's own walks (bvh.rs:315-362, kdtree.rs:101-169).

* Structure: every triangle of an untransformed mesh sits in exactly one leaf of its tree, with its
  object; instanced meshes have their BLAS; every child box contains what it bounds (the f32
  boxes are rounded outward, so the f64 slab test on them never culls a primitive inside); the
  walk stack need is within wbvh::STACK.
* Rays: lumo's walks and the wide walk test the same triangles with the same watertight test, so
  they agree on t, kind and object except where lumo's kd walk skips a hit: its leaf intervals clip
  the triangle test (t <= the leaf's exit), which misses grazing hits on flat boxes (the Cornell
  walls, the floor under a box: a ray from inside the box escapes).  On those rays the wide walk
  is closer (or hits where lumo misses), never farther; at equal t (coincident surfaces) the two
  walks may keep different triangles.  The bound on how many rays differ is stated below.
"""
import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from lumo_amd import scenes
from lumo_amd.procedural import torus_knot_tube
from scenes import material_zoo
from test_gpu_scale import _closest_rays, _visibility_rays
from test_instances_lights import light_scene, sphere_scene

NONE = -(1 << 31)
KDMESH, RECT, TRI, SPHERE = 0, 1, 2, 3


def _scene(name):
    if name == "cornell":
        return L.Scene.cornell_box(), (278.0, 273.0, -800.0)
    if name == "caustics":
        return scenes.caustics(), (0.0, 0.0, 2.0)
    if name == "zoo":
        return material_zoo(), (0.0, 0.0, 0.0)
    if name == "small_dragon":
        return scenes.dragon(torus_knot_tube(300, 12)), (0.0, 0.0, 0.0)
    if name == "tri_lights":
        return light_scene("triangles"), (0.0, 0.5, 4.0)
    if name == "instanced_rect":
        return light_scene("instanced_rect"), (0.0, 0.5, 4.0)
    if name == "spheres":
        return sphere_scene(env=True), (0.0, 0.3, 4.0)
    if name == "lights_only":  # the objects' tree is empty (root NONE)
        sc = L.Scene()
        v, f = torus_knot_tube(100, 8)
        sc.add_mesh(v, f, L.Material.light(L.Spectrum.from_rgb(1.0, 0.8, 0.6), scale=0.5), light=True)
        return sc, (0.0, 0.0, 3.0)
    from lumo_amd.procedural import bistro_standin
    return scenes.bistro(bistro_standin(groups=40, lamps=64, n=4)), (-16.0, 5.0, -1.0)


NAMES = ["cornell", "caustics", "zoo", "small_dragon", "tri_lights", "instanced_rect", "spheres", "bistro_small",
         "lights_only"]


def _leaves(acc, root):
    """(node, child slot, leaf ref) of every leaf reachable from root (root itself may be a leaf)."""
    out, seen = [], set()
    if root == NONE:
        return out, seen
    if root < 0:
        return [(None, None, root)], seen
    stack = [root]
    while stack:
        i = stack.pop()
        assert i not in seen, "a node reached twice: not a tree"
        seen.add(i)
        nd = acc["nodes"][i]
        assert 2 <= nd["n"] <= 4 or (nd["n"] >= 1 and i == root)
        for k in range(nd["n"]):
            r = int(nd["ref"][k])
            if r >= 0:
                stack.append(r)
            else:
                out.append((i, k, r))
    return out, seen


def _box(nd, k):
    return nd["lo"][:, k].astype(np.float64), nd["hi"][:, k].astype(np.float64)


@pytest.mark.parametrize("name", NAMES)
def test_wide_structure(name):
    sc, _ = _scene(name)
    d = sc.build().desc()
    acc = O.wide_export(d)
    assert acc["ok"] and 0 <= acc["stack"] <= 64
    objs = np.ctypeslib.as_array(d.objects, shape=(d.num_objects,)) if d.num_objects else []
    lights = np.ctypeslib.as_array(d.lights, shape=(d.num_lights,))
    tv = acc["tv"]
    reached = set()
    for space, (root, table, blas) in enumerate([(acc["obj_root"], objs, acc["obj_blas"]),
                                                 (acc["light_root"], lights, acc["light_blas"])]):
        leaves, seen = _leaves(acc, root)
        reached |= seen
        got = {}
        for node, k, r in leaves:
            x = ~r
            cnt, first = x & 15, x >> 4
            if cnt == 0:  # object leaf: a sphere or an instance
                o = table[first]
                assert o["type"] == SPHERE or o["xform"] >= 0
                if o["type"] != SPHERE:
                    b = int(blas[first])
                    assert b != NONE
                    bl, bseen = _leaves(acc, b)
                    reached |= bseen
                    tris = sorted(int(acc["tri"][(~br >> 4) + j]) for _, _, br in bl for j in range((~br) & 15))
                    n = 1 if o["type"] == TRI else o["num_tris"]
                    assert tris == list(range(o["tri_base"], o["tri_base"] + n))
                continue
            assert 1 <= cnt <= 15
            if node is not None:  # the child box contains the leaf's triangles (exactly, in f64)
                lo, hi = _box(acc["nodes"][node], k)
                v = tv[first:first + cnt, :9].reshape(-1, 3)
                assert (v >= lo).all() and (v <= hi).all()
            for j in range(first, first + cnt):
                t, o = int(acc["tri"][j]), int(acc["obj"][j])
                assert t not in got, "a triangle in two leaves"
                got[t] = o
        want = {}
        for i, o in enumerate(table):
            if o["xform"] < 0 and o["type"] != SPHERE:
                n = 1 if o["type"] == TRI else o["num_tris"]
                for t in range(o["tri_base"], o["tri_base"] + n):
                    want[t] = i
        assert got == want, f"space {space}: leaves do not hold exactly the untransformed triangles"
        # records hold the scene's vertices
        vtx = np.ctypeslib.as_array(d.vertices, shape=(d.num_vertices, 3))
        tris = np.ctypeslib.as_array(d.triangles, shape=(d.num_triangles,))
        for node, k, r in leaves[:50]:
            x = ~r
            for j in range((x >> 4), (x >> 4) + (x & 15)):
                np.testing.assert_array_equal(tv[j, :9].reshape(3, 3), vtx[tris["v"][acc["tri"][j]]])
    assert reached == set(range(len(acc["nodes"]))), "unreachable nodes"
    # interior children: every box of the child node lies inside the parent's child box
    for i, nd in enumerate(acc["nodes"]):
        for k in range(nd["n"]):
            r = int(nd["ref"][k])
            if r >= 0:
                lo, hi = _box(nd, k)
                ch = acc["nodes"][r]
                for j in range(ch["n"]):
                    clo, chi = _box(ch, j)
                    assert (clo >= lo).all() and (chi <= hi).all()


def _compare(d, o, dirs, lights=None):
    a = O.trace(d, o, dirs, lights)
    b = O.trace(d, o, dirs, lights, accel=1)
    same = ((a[0] == b[0]) | (np.isinf(a[0]) & np.isinf(b[0]))) & (a[1] == b[1]) & (a[2] == b[2])
    return a, b, same


# fraction of rays allowed to differ (measured: <= 0.25 % closest, <= 0.1 % visibility on these
# ray sets; the bound leaves room for other seeds)
BOUND = 0.005


@pytest.mark.parametrize("name", NAMES)
def test_wide_matches_lumo_except_kd_misses(name):
    sc, eye = _scene(name)
    d = sc.build().desc()
    o, dirs = _closest_rays(d, eye, 1 << 15, 21)
    a, b, same = _compare(d, o, dirs)
    bad = ~same
    assert bad.mean() <= BOUND, bad.mean()
    # where they differ, the wide walk found a closer accepted hit (or one where lumo found none), or
    # the same t on another triangle (a tie between coincident surfaces, e.g. a lamp on a facade:
    # each walk keeps the first it finds)
    assert (b[0][bad] <= a[0][bad]).all()
    o, dirs, li = _visibility_rays(d, 1 << 15, 22)
    a, b, same = _compare(d, o, dirs, li)
    assert (~same).mean() <= BOUND, (~same).mean()


def _image(bufs, tasks, W, H):
    f = L.Film(W, H)
    for t, b in zip(tasks, bufs):
        f.add_tile(t, b)
    return f.rgb()


def _tile_diffs(A, B):
    """Per 16x16 tile and channel, the mean of A - B.  lumo's film clips every sample's filter to
    its own tile (tile.rs:74-83), so tiles are independent estimates: their spread gives the
    standard error of the mean difference."""
    H, W, _ = A.shape
    return (A - B).reshape(H // 16, 16, W // 16, 16, 3).mean(axis=(1, 3)).reshape(-1, 3)


def test_wide_image_matches_lumo_cornell():
    """C0 (Cornell 256^2 @ 16) rendered by the oracle on both structures with the same sample
    streams (wavefront order, 2 seeds), so the images differ only by the paths the two walks send
    apart.  The light is coplanar with the ceiling (cornell_box.rs:48-60): where a ray's t on the
    light is an ulp below its t on the ceiling, the wide walk returns the light (scene.rs's rule: a
    light in front of the object), while lumo's kd walk of the light's flat box clips that hit and
    returns the ceiling.  Tolerances: the frame's per-channel mean within 3 % (the
    wide image is ~1.7 % brighter, from the tiles that show the light), the other tiles' mean within
    0.1 % (measured ~0.005 %, the BSDF-sampled rays that reach the light)."""
    sc = L.Scene.cornell_box()
    cam = L.Camera.cornell_box((256, 256))
    for seed in (1, 2):
        tasks = L.make_tasks(256, 256, 16, seed)
        a, _, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
        b, _, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8, accel=1)
        A, B = _image(a, tasks, 256, 256), _image(b, tasks, 256, 256)
        light = (np.maximum(A, B).reshape(16, 16, 16, 16, 3).max(axis=(1, 3, 4)) > 10.0).reshape(-1)
        assert 0 < light.sum() < 40
        rel = np.abs(B.mean(axis=(0, 1)) - A.mean(axis=(0, 1))) / A.mean(axis=(0, 1))
        assert np.all(rel < 0.03), rel
        ta = A.reshape(16, 16, 16, 16, 3).mean(axis=(1, 3)).reshape(-1, 3)[~light].mean(0)
        tb = B.reshape(16, 16, 16, 16, 3).mean(axis=(1, 3)).reshape(-1, 3)[~light].mean(0)
        assert np.all(np.abs(tb - ta) / ta < 1e-3), (ta, tb)


def test_wide_image_matches_lumo_bistro():
    """The C3 scene (Bistro stand-in, full size) at 96 x 64 @ 8 spp, paired as above (no coplanar
    emitters: the lamps sit 0.02 in front of the facades): per-channel means within 0.1 %."""
    sc = scenes.bistro().build()
    cam = scenes.bistro_camera((96, 64))
    tasks = L.make_tasks(96, 64, 8, 3)
    a, _, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    b, _, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8, accel=1)
    A, B = _image(a, tasks, 96, 64), _image(b, tasks, 96, 64)
    ma, mb = A.mean(axis=(0, 1)), B.mean(axis=(0, 1))
    assert np.all(np.abs(mb - ma) / ma < 1e-3), (ma, mb)
