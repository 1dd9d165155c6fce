"""Host-side scene/camera/task construction (CPU only): BVH and kd-tree invariants
(kdtree_tests.rs:83-130 'splits'/'contains'), alias table, task generation (renderer.rs:179-204)
and camera matrices."""
import ctypes as C

import numpy as np
import pytest

import lumo_amd as L
from lumo_amd import _ffi
from lumo_amd.dist import shard_tasks, tiles_per_batch
from pyref import Xorshift

# kdtree_tests.rs:161-194: the Cornell tall-box mesh ("cube"), 5 quads fan-split into 2 triangles
CUBE_V = [(130, 165, 65), (82, 165, 225), (240, 165, 272), (290, 165, 114), (290, 0, 114), (290, 165, 114),
          (240, 165, 272), (240, 0, 272), (130, 0, 65), (130, 165, 65), (290, 165, 114), (290, 0, 114),
          (82, 0, 225), (82, 165, 225), (130, 165, 65), (130, 0, 65), (240, 0, 272), (240, 165, 272),
          (82, 165, 225), (82, 0, 225)]
CUBE_F = [f for i in range(5) for f in ((4 * i, 4 * i + 1, 4 * i + 2), (4 * i, 4 * i + 2, 4 * i + 3))]


def tiny_light(scene):
    white = L.Spectrum.from_rgb(1.0, 1.0, 1.0)
    scene.add_rectangle((-1e4, 1e4, -1e4), (-1e4 + 1, 1e4, -1e4), (-1e4 + 1, 1e4, -1e4 + 1),
                        L.Material.light(white), light=True)


def arr(ptr, n):
    return [ptr[i] for i in range(n)]


def verts(d):
    return np.ctypeslib.as_array(d.vertices, shape=(d.num_vertices * 3,)).reshape(-1, 3)


def tri_boxes(d, ob):
    v = verts(d)
    out = []
    for k in range(ob.num_tris):
        t = d.triangles[ob.tri_base + k]
        p = v[list(t.v)]
        out.append((p.min(0), p.max(0)))
    return out


def aabb_contains_triangle(bmin, bmax, tb):
    """kdtree_tests.rs:9-24"""
    tmin, tmax = tb
    for a in range(3):
        intersect = tmin[a] < bmax[a] and bmin[a] < tmax[a]
        planar = tmin[a] == tmax[a] and (tmin[a] == bmin[a] or tmax[a] == bmax[a])
        if not (intersect or planar):
            return False
    return True


def kd_leaves(d, ob):
    """Walk the object's kd-tree from its boundary, splitting bounds like AaBoundingBox::split."""
    out = []
    stack = [(ob.kd_root, np.array(ob.bmin[:]), np.array(ob.bmax[:]))]
    while stack:
        idx, bmin, bmax = stack.pop()
        if idx < 0:
            continue
        n = d.kd_nodes[idx]
        if not n.leaf:
            lmax, rmin = bmax.copy(), bmin.copy()
            lmax[n.axis] = n.point
            rmin[n.axis] = n.point
            stack.append((n.right, rmin, bmax))
            stack.append((idx + 1, bmin, lmax))
        else:
            items = [d.kd_items[ob.item_base + n.first + k] for k in range(n.count)]
            out.append((bmin, bmax, items))
    return out


def all_kd_objects(d):
    return [d.objects[i] for i in range(d.num_objects)] + [d.lights[i] for i in range(d.num_lights)]


@pytest.fixture(scope="module")
def cornell():
    s = L.Scene.cornell_box()
    return s, s.desc()


@pytest.fixture(scope="module")
def cube():
    s = L.Scene()
    s.add_mesh(np.array(CUBE_V, dtype=float), CUBE_F, L.Material.lambertian(L.Spectrum.from_rgb(0.5, 0.5, 0.5)))
    tiny_light(s)
    return s, s.desc()


@pytest.mark.parametrize("which", ["cornell", "cube"])
def test_kd_splits_and_contains(which, request):
    _, d = request.getfixturevalue(which)
    for ob in all_kd_objects(d):
        boxes = tri_boxes(d, ob)
        found = set()
        for bmin, bmax, items in kd_leaves(d, ob):
            assert all(aabb_contains_triangle(bmin, bmax, boxes[i]) for i in items)
            for i, tb in enumerate(boxes):
                assert not aabb_contains_triangle(bmin, bmax, tb) or i in items
            found |= set(items)
        assert found == set(range(ob.num_tris))


@pytest.mark.parametrize("which", ["cornell", "cube"])
def test_bvh_leaves_partition_and_nest(which, request):
    _, d = request.getfixturevalue(which)
    for nodes, n_nodes, items, objs, n_objs in (
            (d.object_nodes, d.num_object_nodes, d.object_items, d.objects, d.num_objects),
            (d.light_nodes, d.num_light_nodes, d.light_items, d.lights, d.num_lights)):
        seen = []

        def walk(i, pmin, pmax):
            n = nodes[i]
            bmin, bmax = np.array(n.bmin[:]), np.array(n.bmax[:])
            assert np.all(bmin >= pmin) and np.all(bmax <= pmax)
            if n.count > 0:
                for k in range(n.count):
                    o = objs[items[n.first + k]]
                    assert np.all(np.array(o.bmin[:]) >= bmin) and np.all(np.array(o.bmax[:]) <= bmax)
                    seen.append(items[n.first + k])
            else:
                walk(i + 1, bmin, bmax)  # left child = i + 1 (bvh.rs:324-360)
                if n.right >= 0:
                    walk(n.right, bmin, bmax)

        if n_nodes:
            walk(0, np.full(3, -np.inf), np.full(3, np.inf))
        assert sorted(seen) == list(range(n_objs))


def test_alias_table(cornell):
    _, d = cornell
    n = d.num_lights
    prob = np.array(arr(d.alias_prob, n))
    pdf = np.array(arr(d.alias_pdf, n))
    idx = np.array(arr(d.alias_idx, n))
    assert np.all((prob >= 0) & (prob <= 1)) and np.all((idx >= 0) & (idx < n))
    np.testing.assert_allclose(pdf.sum(), 1.0, rtol=1e-12)
    # the table reproduces the pdf: P(i) = (prob_i + sum_{j: idx_j = i} (1 - prob_j)) / n
    rec = prob.copy()
    for j in range(n):
        rec[idx[j]] += 1.0 - prob[j]
    np.testing.assert_allclose(rec / n, pdf, atol=1e-12)


def test_alias_table_many_lights():
    s = L.Scene()
    white = L.Spectrum.from_rgb(1.0, 1.0, 1.0)
    areas = [1.0, 2.0, 4.0, 0.5, 3.0]
    for k, a in enumerate(areas):
        x = 10.0 * k
        s.add_rectangle((x, 0, 0), (x + a, 0, 0), (x + a, 0, 1), L.Material.light(white), light=True)
    d = s.desc()
    n = d.num_lights
    pdf = np.array(arr(d.alias_pdf, n))
    area = np.array([d.lights[i].area for i in range(n)])
    # same emitter spectrum: power ∝ area (bvh.rs:105-191)
    np.testing.assert_allclose(pdf, area / area.sum(), rtol=1e-12)
    prob, idx = np.array(arr(d.alias_prob, n)), np.array(arr(d.alias_idx, n))
    rec = prob.copy()
    for j in range(n):
        rec[idx[j]] += 1.0 - prob[j]
    np.testing.assert_allclose(rec / n, pdf, atol=1e-12)


@pytest.mark.parametrize("w,h,spp", [(32, 32, 8), (40, 23, 300), (1024, 1024, 1024), (17, 1, 1)])
def test_make_tasks_order_and_seeds(w, h, spp):
    seed = 0xC0FFEE
    tasks = L.make_tasks(w, h, spp, seed)
    tx, ty = (w + 15) // 16, (h + 15) // 16
    batches = (spp + 255) // 256
    assert len(tasks) == tx * ty * batches
    rng = Xorshift(seed)
    i = 0
    for b in range(batches):
        for y in range(ty):
            for x in range(tx):
                t = tasks[i]
                assert (t.px_min[0], t.px_min[1]) == (16 * x, 16 * y)
                assert (t.px_max[0], t.px_max[1]) == (min(16 * x + 16, w), min(16 * y + 16, h))
                assert t.batch == b and t.total_samples == spp
                assert t.samples == min(256, spp - 256 * b)
                assert t.seed == rng.gen_u64()
                i += 1


def test_make_tasks_empty():
    assert L.lib().lumo_make_tasks(0, 16, 4, 1, None, 0) == 0
    assert L.lib().lumo_make_tasks(16, 16, 0, 1, None, 0) == 0


@pytest.mark.parametrize("ws", [1, 2, 3, 8])
def test_shards_cover_each_task_once(ws):
    w, h, spp = 80, 48, 600
    tasks = L.make_tasks(w, h, spp, 7)
    seen = []
    tpb = tiles_per_batch(w, h)
    for r in range(ws):
        mine = shard_tasks(tasks, w, h, r, ws)
        tiles = {(t.px_min[0], t.px_min[1]) for t in mine}
        # every batch of a tile lands on the same rank
        assert all(sum(1 for t in mine if (t.px_min[0], t.px_min[1]) == k) == (spp + 255) // 256 for k in tiles)
        seen += [t.seed for t in mine]
    assert sorted(seen) == sorted(t.seed for t in tasks)
    assert tpb == 5 * 3
    with pytest.raises(ValueError):
        shard_tasks(tasks, w, h, ws, ws)


def _mat(m):
    return np.array(m[:]).reshape(4, 4)


def test_camera_matrices():
    cam = L.Camera.cornell_box((64, 48))
    d = cam.desc
    for pair in (d.world_to_camera, d.screen_to_raster, d.camera_to_screen):
        np.testing.assert_allclose(_mat(pair[0]) @ _mat(pair[1]), np.eye(4), atol=1e-9)
    w2c = _mat(d.world_to_camera[0])
    o = w2c @ np.array([278.0, 273.0, -800.0, 1.0])  # camera.rs:139-148 origin
    np.testing.assert_allclose(o[:3], 0.0, atol=1e-9)
    f = w2c @ np.array([278.0, 273.0, 0.0, 1.0])  # looking towards
    np.testing.assert_allclose(f[:2], 0.0, atol=1e-9)
    assert abs(f[2]) == pytest.approx(800.0)
    assert (d.width, d.height) == (64, 48)
    assert d.filter_radius == 1.5 and d.filter_sigma == 0.375  # filter.rs:20-24


def test_camera_rejects_bad_params():
    b = L.Camera.builder()
    b.p.origin[:] = [0, 0, 0]
    b.p.towards[:] = [0, 0, 0]
    with pytest.raises(Exception):
        b.build()
    with pytest.raises(Exception):
        L.Camera.builder().vfov(180.0).build()
    with pytest.raises(Exception):
        L.Camera.builder().resolution((0, 10)).build()


def test_scene_without_light_fails():
    s = L.Scene()
    s.add_mesh(np.array(CUBE_V, dtype=float), CUBE_F, L.Material.lambertian(L.Spectrum.from_rgb(0.5, 0.5, 0.5)))
    with pytest.raises(ValueError):
        s.build()


def test_builder_rejects_bad_mesh():
    s = L.Scene()
    with pytest.raises(Exception):
        s.add_mesh(np.zeros((3, 3)), [(0, 1, 5)], L.Material.lambertian(L.Spectrum.from_rgb(0.5, 0.5, 0.5)))
    with pytest.raises(Exception):
        s.add_mesh(np.zeros((3, 3)), [(0, 1)], L.Material.lambertian(L.Spectrum.from_rgb(0.5, 0.5, 0.5)))
