"""GPU traversal parity: lumo_trace (closest hit = Scene::hit, visibility = Scene::hit_light)
vs the oracle on the same rays.  Bar: bit-exact t, kind and object index."""
import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from test_oracle import disk_scene, sphere_points, unit_cube_scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = L.Device(0)
    yield d
    d.close()


def _rays_in_box(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform([1, 1, 1], [555, 548, 558], size=(n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d


def _cmp(dev, scene, o, d, lights=None):
    dev.upload(scene)
    g = dev.trace(o, d, lights)
    r = O.trace(scene.desc(), o, d, lights)
    np.testing.assert_array_equal(g[0], r[0])
    np.testing.assert_array_equal(g[1], r[1])
    np.testing.assert_array_equal(g[2], r[2])
    return g


def test_closest_cornell(dev):
    o, d = _rays_in_box(200000, 1)
    t, kind, _, prim = _cmp(dev, L.Scene.cornell_box(), o, d)
    assert np.mean(kind > 0) > 0.8  # the box is open towards the camera (z = 0)
    assert np.all(prim[kind == 1] >= 0)


def test_visibility_cornell(dev):
    sc = L.Scene.cornell_box()
    o, _ = _rays_in_box(100000, 2)
    # aim at points on the light rectangle (cornell_box.rs: y = 548.8 ceiling light)
    rng = np.random.default_rng(3)
    tgt = np.stack([rng.uniform(213, 343, len(o)), np.full(len(o), 548.7), rng.uniform(227, 332, len(o))], 1)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    t, kind, _, _ = _cmp(dev, sc, o, d, lights=np.zeros(len(o), dtype=np.int32))
    assert 0.05 < np.mean(kind == 2) < 0.99


def test_property_scenes(dev):
    s = unit_cube_scene()
    xo = sphere_points(10000, 3, 5.0)
    xo = xo[xo[:, 1] > -0.1]
    d = -xo / np.linalg.norm(xo, axis=1, keepdims=True)
    _, kind, _, _ = _cmp(dev, s, xo, d)
    assert np.all(kind == 1)
    _cmp(dev, disk_scene(), np.array([(0.0, 0.0, 0.0), (0.0, 3.0, 0.0)]),
         np.array([(0.0, 1.0, 0.0), (0.0, -1.0, 0.0)]), lights=np.array([0, 0]))


def test_trace_rejects_bad_light(dev):
    dev.upload(L.Scene.cornell_box())
    with pytest.raises(Exception):
        dev.trace(np.zeros((1, 3)), np.array([(0.0, 1.0, 0.0)]), lights=np.array([5]))


def one_child_light_scene():
    """Triangle lights whose light BVH has interior nodes without a right child: five concentric
    triangles share a bounding-box centre, so every SAH cost of their node is NaN (0 x INF,
    bvh/node.rs:176-190), the partition puts all of them on the left (node.rs:146-168) and the
    chain continues down to the Morton depth.  (The shape behind round 2's fault in a rejected
    traversal variant.)"""
    s = L.Scene()
    v, f = [], []
    for sc in (0.2, 0.4, 0.6, 0.8, 1.0):
        b = len(v)
        v += [(-sc, 2.0, -sc), (sc, 2.0, -sc), (0.0, 2.0, sc)]
        f.append((b, b + 2, b + 1))
    for x in (-3.0, 3.0):
        b = len(v)
        v += [(x - 0.3, 2.5, -0.3), (x + 0.3, 2.5, -0.3), (x, 2.5, 0.3)]
        f.append((b, b + 2, b + 1))
    s.add_mesh(np.array(v, dtype=float), f, L.Material.light(L.named_spectrum("WHITE")), light=True)
    s.add_rectangle((-5, -1, 5), (5, -1, 5), (5, -1, -5), L.Material.diffuse(L.Spectrum.from_srgb(200, 200, 200)))
    s.build()
    return s, np.array(v, dtype=float).reshape(-1, 3, 3)


def test_light_bvh_without_right_child(dev):
    s, tris = one_child_light_scene()
    d = s.desc()
    nodes = [d.light_nodes[i] for i in range(d.num_light_nodes)]
    assert sum(1 for n in nodes if n.count == 0 and n.right < 0) >= 8
    rng = np.random.default_rng(7)
    n = 100000
    o = np.stack([rng.uniform(-4, 4, n), rng.uniform(-0.9, 1.9, n), rng.uniform(-2, 2, n)], 1)
    # closest: random upward directions (lights, the floor's back, misses)
    dd = rng.normal(size=(n, 3))
    dd[:, 1] = np.abs(dd[:, 1]) + 0.3
    dd /= np.linalg.norm(dd, axis=1, keepdims=True)
    _, kind, obj, _ = _cmp(dev, s, o, dd)
    assert np.mean(kind == 2) > 0.02
    assert len(np.unique(obj[kind == 2])) >= 3
    # visibility towards a point on each light (the concentric ones occlude each other)
    li = rng.integers(0, d.num_lights, n).astype(np.int32)
    bary = rng.dirichlet([1, 1, 1], n)
    # light i is face i of the mesh (parser order); aim at a point of that triangle
    tgt = np.einsum("nk,nkj->nj", bary, tris[li])
    dv = tgt - o
    dv /= np.linalg.norm(dv, axis=1, keepdims=True)
    t, kind, _, _ = _cmp(dev, s, o, dv, lights=li)
    assert 0.5 < np.mean(kind == 2) < 1.0  # coplanar lights do not occlude each other (t_max = t - 1e-10)
