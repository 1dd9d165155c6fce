"""GPU parity at the benchmarked scale and over every kernel variant the bench can select.

* The full-size C2 (dragon.rs + the 871 414-triangle stand-in, kd stack class 48) and C3 (Bistro
  stand-in, ~2.8 M triangles in 400 groups, 2 048 triangle lights, class 24) scenes exactly as
  bench.py builds them: lumo_trace on >= 1 M rays, closest hit (Scene::hit, scene.rs:119-147)
  and light visibility (Scene::hit_light, scene.rs:165-189), against the oracle, bit-exact in
  t / kind / object and in the traversal counters (AABB / kd / triangle tests, the roofline's
  inputs); per-path parity of two 16x16 tiles at each bench camera (k_closest / k_shade /
  k_shadow of that stack class, kdtree.rs:101-169 + bvh.rs:315-362 semantics).
* Cornell and the small dragon over every stack class >= the scene's need x LDS staging on/off
  x lean/full feature kernels (options stack_class, lds_staging, full_kernels):
  per-path parity and tile parity for each instantiation, with lumo_scene_info confirming the
  variant that ran.
"""
import os

import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from lumo_amd import _ffi, scenes
from lumo_amd.procedural import torus_knot_tube
from parity import gpu_paths, oracle_threads

pytestmark = pytest.mark.gpu
SEED = 0x5EED1234
CLASSES = [4, 8, 16, 24, 32, 48, 64]  # launch.h STACK_CLASSES


@pytest.fixture(scope="module")
def dev():
    d = L.Device(0)
    yield d
    d.close()


@pytest.fixture(scope="module")
def c2():
    return scenes.dragon().build()


@pytest.fixture(scope="module")
def c3():
    return scenes.bistro().build()


def _arrays(desc):
    v = np.ctypeslib.as_array(desc.vertices, shape=(desc.num_vertices, 3))
    tris = np.ctypeslib.as_array(desc.triangles, shape=(desc.num_triangles,))
    return v, tris


def _closest_rays(desc, eye, n, seed):
    """Half camera-like rays from the bench eye, half rays from random points of the scene's
    bounds in random directions (the secondary-ray mix)."""
    rng = np.random.default_rng(seed)
    v, _ = _arrays(desc)
    lo, hi = v.min(0), v.max(0)
    m = n // 2
    o1 = np.repeat(np.asarray(eye, dtype=np.float64)[None], m, 0)
    d1 = (rng.uniform(lo, hi, size=(m, 3)) - o1)
    o2 = rng.uniform(lo, hi, size=(n - m, 3))
    d2 = rng.normal(size=(n - m, 3))
    o, d = np.concatenate([o1, o2]), np.concatenate([d1, d2])
    return o, d / np.linalg.norm(d, axis=1, keepdims=True)


def _visibility_rays(desc, n, seed):
    """Rays from random points of the bounds towards a random point of a random light
    (triangle lights: a uniform barycentric point; rectangles: a uniform point; the environment
    sphere: a random direction)."""
    rng = np.random.default_rng(seed)
    v, tris = _arrays(desc)
    lights = np.ctypeslib.as_array(desc.lights, shape=(desc.num_lights,))
    lo, hi = v.min(0), v.max(0)
    o = rng.uniform(lo, hi, size=(n, 3))
    li = rng.integers(0, desc.num_lights, size=n).astype(np.int32)
    d = rng.normal(size=(n, 3))  # the environment sphere: any direction
    is_tri = lights["type"][li] == 2  # LUMO_OBJ_TRIANGLE
    tb = lights["tri_base"][li[is_tri]]
    vi = np.stack([tris["v"][tb][:, k] for k in range(3)], 1)
    a, b, c = v[vi[:, 0]], v[vi[:, 1]], v[vi[:, 2]]
    u = rng.uniform(size=(len(tb), 2))
    s = np.sqrt(u[:, :1])
    p = (1 - s) * a + s * (1 - u[:, 1:]) * b + s * u[:, 1:] * c
    d[is_tri] = p - o[is_tri]
    is_rect = lights["type"][li] == 1  # LUMO_OBJ_RECTANGLE: origin + u b0 + v b1
    lr = lights[li[is_rect]]
    u = rng.uniform(size=(len(lr), 2))
    d[is_rect] = lr["origin"] + u[:, :1] * lr["b0"] + u[:, 1:] * lr["b1"] - o[is_rect]
    return o, d / np.linalg.norm(d, axis=1, keepdims=True), li


def _trace_cmp(dev, sc, o, d, lights=None):
    dev.upload(sc)
    before = dev.stats()
    g = dev.trace(o, d, lights)
    after = dev.stats()
    t, kind, obj, cnt = O.trace(sc.desc(), o, d, lights)
    np.testing.assert_array_equal(g[0], t)
    np.testing.assert_array_equal(g[1], kind)
    np.testing.assert_array_equal(g[2], obj)
    k = 0 if lights is None else 1
    got = [after.aabb_tests[k] - before.aabb_tests[k], after.kd_nodes[k] - before.kd_nodes[k],
           after.tri_tests[k] - before.tri_tests[k]]
    assert got == [cnt.aabb_tests, cnt.kd_nodes, cnt.tri_tests]
    return g


@pytest.mark.parametrize("which", ["c2", "c3"])
def test_trace_closest_full_scale(dev, which, request):
    sc = request.getfixturevalue(which)
    eye = (0.0, 0.0, 0.0) if which == "c2" else (-16.0, 5.0, -1.0)
    o, d = _closest_rays(sc.desc(), eye, 1 << 20, 11)
    g = _trace_cmp(dev, sc, o, d)
    info = dev.scene_info()
    assert info.stack_class == (48 if which == "c2" else 24)
    if which == "c2":  # the dragon's top kd treelets are walked from LDS (C3's TOP set is full)
        assert info.top_kd_nodes > 1000
    assert np.mean(g[1] > 0) > 0.3


@pytest.mark.parametrize("which", ["c2", "c3"])
def test_trace_visibility_full_scale(dev, which, request):
    sc = request.getfixturevalue(which)
    o, d, li = _visibility_rays(sc.desc(), 1 << 20, 12)
    g = _trace_cmp(dev, sc, o, d, lights=li)
    assert 0.01 < np.mean(g[1] == 2) < 0.99


def _paths(dev, sc, cam, task):
    dev.upload(sc, cam)
    g = gpu_paths(dev, task)
    o = O.trace_paths(sc.desc(), cam.desc, task)
    for k in ("depth", "raster", "lam", "radiance", "delta"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)
    return g


@pytest.mark.parametrize("which", ["c2", "c3"])
def test_paths_full_scale_bench_camera(dev, which, request):
    """Two tiles of the bench frame (1920x1080, the bench camera): one central, one off-centre."""
    sc = request.getfixturevalue(which)
    cam = scenes.default_camera((1920, 1080)) if which == "c2" else scenes.bistro_camera((1920, 1080))
    tasks = L.make_tasks(1920, 1080, 4, SEED)
    tiles_x = 1920 // 16
    for ty, tx in ((34, 60), (20, 35)):
        g = _paths(dev, sc, cam, tasks[ty * tiles_x + tx])
        assert (g["depth"] > 1).any()


# ---------------------------------------------------------------------------- kernel variants
@pytest.fixture
def variant_env(dev):
    yield
    dev.set_option("stack_class", 0).set_option("full_kernels", 0).set_option("lds_staging", 1)


def _variant_scene(name):
    if name == "cornell":
        return L.Scene.cornell_box(), L.Camera.cornell_box((48, 48)), L.make_tasks(48, 48, 8, SEED)
    sc = scenes.dragon(torus_knot_tube(300, 12))
    return sc, scenes.default_camera((48, 32)), L.make_tasks(48, 32, 8, SEED)


@pytest.mark.parametrize("full", [0, 1])
@pytest.mark.parametrize("lds", [1, 0])
@pytest.mark.parametrize("cls", CLASSES)
@pytest.mark.parametrize("name", ["cornell", "small_dragon"])
def test_kernel_variants(dev, variant_env, name, cls, lds, full):
    sc, cam, tasks = _variant_scene(name)
    sc.build()
    dev.set_option("stack_class", cls).set_option("full_kernels", full).set_option("lds_staging", lds)
    dev.upload(sc, cam)
    info = dev.scene_info()
    if info.stack_class != cls:
        # the override never goes below the scene's need (kdtree.rs:110 stack bound)
        assert info.stack_class > cls
        pytest.skip(f"stack class {cls} below the scene's need ({info.stack_class})")
    assert (info.lds_bytes > 0) == (lds == 1 and name == "cornell")  # the dragon mesh exceeds 48 KiB
    assert info.full_kernels == (1 if (full or name == "small_dragon") else 0)
    g = gpu_paths(dev, tasks[1])
    o = O.trace_paths(sc.desc(), cam.desc, tasks[1])
    for k in ("depth", "raster", "lam", "radiance", "delta"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)
    sub = list(tasks)[:6]
    bufs, res = dev.render_tasks(sub)
    obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, sub, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)


@pytest.mark.parametrize("fused,tail,pipe", [(1, 0, 0), (1, 300, 0), (0, 1 << 30, 0), (1, 0, 1), (1, 0, 2), (1, 0, 3),
                                             (0, 0, 1), (0, 1 << 18, 1)])
def test_bounce_modes_small_dragon(dev, fused, tail, pipe):
    """The fused bounce kernel and the tail kernel on an instanced glass mesh (feature class 1,
    no LDS staging, deep kd stack): paths and tiles equal the oracle's."""
    dev.set_option("fused", fused).set_option("tail_below", tail).set_option("pipeline", pipe)
    try:
        sc, cam, tasks = _variant_scene("small_dragon")
        sc.build()
        dev.upload(sc, cam)
        g = gpu_paths(dev, tasks[1])
        o = O.trace_paths(sc.desc(), cam.desc, tasks[1])
        for k in ("depth", "raster", "lam", "radiance", "delta"):
            np.testing.assert_array_equal(g[k], o[k], err_msg=k)
        sub = list(tasks)[:6]
        bufs, res = dev.render_tasks(sub)
        obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, sub, O.WAVEFRONT, 8)
        for b, ob, r, orr in zip(bufs, obufs, res, ores):
            np.testing.assert_array_equal(b, ob)
            assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
    finally:
        dev.set_option("fused", -1).set_option("tail_below", 1 << 16).set_option("pipeline", 3)


# ---------------------------------------------------------------------------- TOP staging
@pytest.fixture(scope="module")
def mid_bistro():
    from lumo_amd.procedural import bistro_standin
    return scenes.bistro(bistro_standin(groups=48, lamps=160, n=8)).build()


def test_top_staging_selected_for_large_scenes(dev, c3):
    """A scene too large to stage whole (C3) runs its closest-hit and visibility walks with the
    TOP set in LDS: the whole objects BVH, the object records and the top of the lights BVH."""
    dev.upload(c3)
    info = dev.scene_info()
    d = c3.desc()
    assert info.lds_bytes == 0
    assert 0 < info.top_bytes <= 160 * 1024
    assert info.top_object_nodes == d.num_object_nodes
    assert 0 < info.top_light_nodes < d.num_light_nodes


@pytest.mark.parametrize("budget_kb,top", [(0, 0), (8, 1), (20, 1), (None, 1)])
def test_top_staging_budgets(mid_bistro, budget_kb, top):
    """The TOP walk reads node i from LDS when i is below the staged prefix of its BVH and from
    HBM otherwise: with the staged prefix cutting the objects BVH (8 KiB), the lights BVH
    (20 KiB), neither (default) or TOP off, lumo_trace (t / kind / object and the traversal
    counters) and rendered tiles equal the oracle's."""
    opts = {"top_staging": top}
    if budget_kb is not None:
        opts["top_kb"] = budget_kb
    d = L.Device(0, **opts)  # the budget applies at the scene upload
    sc = mid_bistro
    d.upload(sc)
    info = d.scene_info()
    desc = sc.desc()
    if top == 0:
        assert info.top_bytes == 0
    elif budget_kb == 8:
        assert 0 < info.top_object_nodes < desc.num_object_nodes and info.top_light_nodes == 0
    elif budget_kb == 20:
        assert info.top_object_nodes == desc.num_object_nodes and 0 < info.top_light_nodes < desc.num_light_nodes
    else:
        assert info.top_object_nodes == desc.num_object_nodes and info.top_light_nodes == desc.num_light_nodes
    o, dd = _closest_rays(desc, (-16.0, 5.0, -1.0), 1 << 17, 21)
    _trace_cmp(d, sc, o, dd)
    o, dd, li = _visibility_rays(desc, 1 << 17, 22)
    _trace_cmp(d, sc, o, dd, lights=li)
    cam = scenes.bistro_camera((96, 64))
    d.upload(sc, cam)
    tasks = L.make_tasks(96, 64, 4, SEED)[8:14]
    bufs, res = d.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(desc, cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
    d.close()


@pytest.mark.parametrize("k,groups", [(1, 1), (2, 1), (3, 1), (4, 1), (2, 2), (4, 2), (3, 3), (4, 4)])
def test_split_pipeline_passes_in_flight(mid_bistro, k, groups):
    """render_split_pipelined (n_shadow > 1, three-kernel bounces): 1 (sequential) to 4 units of
    (task group, pass) in flight on their own streams and pass sets, with the 12 tasks cut into 1-4
    independent groups; a 9-pass render's tiles, ray and query counts equal the oracle's (a unit
    waits for its group's previous pass's camera, and its ring before bounce RR_DEPTH and before
    its film; set reuse is ordered by stream)."""
    d = L.Device(0, split_pipe=k, split_groups=groups, merge_passes=1)  # one-pass units (merged: below)
    cam = scenes.bistro_camera((64, 48))
    d.upload(mid_bistro, cam)
    assert d.scene_info().n_shadow > 1
    tasks = L.make_tasks(64, 48, 9, SEED)
    before = d.stats()
    bufs, res = d.render_tasks(tasks)
    after = d.stats()
    sch = d.last_schedule()
    d.close()
    # the requested schedule ran (free HBM did not cut the units in flight back)
    if k == 1:
        assert sch.schedule == 0
    else:
        assert (sch.schedule, sch.units_in_flight, sch.task_groups) == (2, k, min(groups, k))
    obufs, ores, cnt = O.render_tasks(mid_bistro.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
    assert after.closest_queries - before.closest_queries == cnt.closest_queries
    assert after.shadow_queries - before.shadow_queries == cnt.shadow_queries


@pytest.mark.parametrize("scene,merge,k,groups", [("bistro", 8, 4, 2), ("bistro", 2, 4, 2), ("bistro", 3, 3, 1),
                                                   ("bistro", 8, 4, 4), ("dragon", 8, 4, 2), ("dragon", 4, 2, 2)])
def test_split_merged_passes(mid_bistro, scene, merge, k, groups):
    """Merged passes in render_split_pipelined: a unit's camera generates the samples of M passes
    into one queue, its first RR_DEPTH bounces run them at once (they read no delta,
    path_trace.rs:60-69), k_split_passes cuts the queue by pass, and each pass runs its remaining
    bounces (the tail kernel included, n_shadow = 1) after the ring before it.  Opt-in (option
    merge_passes; measured slower at C3's share).  9 passes (a ragged last unit),
    M = 2 / 3 / 4 / 8: tiles, ray and query counts equal sequential passes and the oracle's."""
    if scene == "bistro":
        sc, cam = mid_bistro, scenes.bistro_camera((64, 48))
    else:
        sc = scenes.dragon(torus_knot_tube(300, 12)).build()
        cam = scenes.default_camera((64, 48))
    d = L.Device(0, split_pipe=k, split_groups=groups, merge_passes=merge, tail_below=300)
    try:
        d.upload(sc, cam)
        tasks = L.make_tasks(64, 48, 9, SEED)
        before = d.stats()
        bufs, res = d.render_tasks(tasks)
        after = d.stats()
        sch = d.last_schedule()
        assert (sch.schedule, sch.units_in_flight, sch.task_groups) == (2, k, min(groups, k))
        assert sch.merged_passes == merge
        if scene == "dragon":
            assert after.tail_queries > before.tail_queries
        d.set_option("split_pipe", 1)
        seq, seq_res = d.render_tasks(tasks)
        assert d.last_schedule().schedule == 0
    finally:
        d.close()
    obufs, ores, cnt = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    for b, sb, ob, r, sr, orr in zip(bufs, seq, obufs, res, seq_res, ores):
        np.testing.assert_array_equal(b, ob)
        np.testing.assert_array_equal(sb, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
        assert (sr.num_rays, sr.num_queries) == (orr.num_rays, orr.num_queries)
    assert after.closest_queries - before.closest_queries == cnt.closest_queries
    assert after.shadow_queries - before.shadow_queries == cnt.shadow_queries


def test_c3_share_merged_passes(c3):
    """One rank's share of the 8-GPU C3 run (the tiles with tile % 8 == 0 of 1920x1080, 261 k slots
    per pass) at 16 spp with merged passes (merge_passes 8): 4 units of 8 passes in flight in 2 task
    groups.  Every tile, ray and query count equals sequential passes; every 8th tile the oracle's."""
    from lumo_amd.dist import shard_tasks
    W, H, spp = 1920, 1080, 16
    cam = scenes.bistro_camera((W, H))
    tasks = shard_tasks(L.make_tasks(W, H, spp, SEED), W, H, 0, 8)
    d = L.Device(0, merge_passes=8)
    try:
        d.upload(c3, cam)
        bufs, res = d.render_tasks(tasks, max_paths=1 << 23)
        sch = d.last_schedule()
        assert (sch.schedule, sch.units_in_flight, sch.task_groups, sch.merged_passes) == (2, 4, 2, 8)
        d.set_option("split_pipe", 1)
        seq, seq_res = d.render_tasks(tasks, max_paths=1 << 23)
        assert d.last_schedule().schedule == 0
    finally:
        d.close()
    for b, s, r, sr in zip(bufs, seq, res, seq_res):
        np.testing.assert_array_equal(b, s)
        assert (r.num_rays, r.num_queries) == (sr.num_rays, sr.num_queries)
    sub = list(range(0, len(tasks), 8))
    obufs, ores, _ = O.render_tasks(c3.desc(), cam.desc, [tasks[i] for i in sub], O.WAVEFRONT, oracle_threads())
    bad = [i for i, ob in zip(sub, obufs) if not np.array_equal(bufs[i], ob)]
    assert not bad, f"{len(bad)} of {len(sub)} sampled tiles differ, first {bad[:8]}"
    for i, orr in zip(sub, ores):
        assert (res[i].num_rays, res[i].num_queries) == (orr.num_rays, orr.num_queries)


@pytest.mark.parametrize("scene", ["dragon", "bistro"])
def test_ray_sort_matches_oracle(mid_bistro, scene):
    """Ray sorting (option ray_sort): each bounce's closest-hit rays are counting-sorted by direction
    octant and origin cell (scan.h, 12-bit keys) and walked in that order; the hits land at the rays'
    own queue positions, so tiles, ray and query counts equal the oracle's (kdtree.rs:101-169,
    bvh.rs:315-362: the walks themselves are unchanged).  lumo_stats.sorted_bounces shows that the
    sorted walk ran."""
    if scene == "bistro":
        sc, cam = mid_bistro, scenes.bistro_camera((256, 192))
    else:
        sc = scenes.dragon(torus_knot_tube(300, 12)).build()
        cam = scenes.default_camera((256, 192))
    # no tail kernel (every bounce walks through k_closest_q) and one task group (49 k rays per bounce,
    # above the sort minimum of 32 k)
    d = L.Device(0, ray_sort=1, tail_below=0, split_groups=1)
    try:
        d.upload(sc, cam)
        tasks = L.make_tasks(256, 192, 2, SEED)  # 49 k slots per pass: bounces above the sort minimum
        before = d.stats()
        bufs, res = d.render_tasks(tasks)
        after = d.stats()
    finally:
        d.close()
    obufs, ores, cnt = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, oracle_threads())
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
    assert after.closest_queries - before.closest_queries == cnt.closest_queries
    assert after.shadow_queries - before.shadow_queries == cnt.shadow_queries
    assert after.sorted_bounces - before.sorted_bounces > 0


def test_c3_bench_schedule_full_frame(c3):
    """C3 as the bench renders it: the full 1920x1080 Bistro stand-in frame (8 160 tiles, 2.07 M
    slots per pass, n_shadow = 11, the full TOP set) through render_split_pipelined with the
    default 4 units in flight in 2 task groups, at 2 spp.  Every tile, ray and query count equals
    the same frame with sequential passes (split_pipe 1), and every 64th tile equals the oracle's
    (task.rs:25-82 pass order, renderer.rs:179-204 tasks).  Buffers are poisoned (conftest), so a
    unit that read another stream's stale counters or tables would show."""
    W, H, spp = 1920, 1080, 2
    cam = scenes.bistro_camera((W, H))
    tasks = L.make_tasks(W, H, spp, SEED)
    d = L.Device(0)
    try:
        d.upload(c3, cam)
        info = d.scene_info()
        assert info.n_shadow == 11 and info.top_bytes > 0 and info.top_object_nodes == c3.desc().num_object_nodes
        before = d.stats()
        bufs, res = d.render_tasks(tasks, max_paths=1 << 23)
        after = d.stats()
        sch = d.last_schedule()
        assert (sch.schedule, sch.units_in_flight, sch.task_groups, sch.fused) == (2, 4, 2, 0)
        d.set_option("split_pipe", 1)
        seq, seq_res = d.render_tasks(tasks, max_paths=1 << 23)
        assert d.last_schedule().schedule == 0
    finally:
        d.close()
    for b, s, r, sr in zip(bufs, seq, res, seq_res):
        np.testing.assert_array_equal(b, s)
        assert (r.num_rays, r.num_queries) == (sr.num_rays, sr.num_queries)
    sub = list(range(0, len(tasks), 64))
    obufs, ores, _ = O.render_tasks(c3.desc(), cam.desc, [tasks[i] for i in sub], O.WAVEFRONT, oracle_threads())
    bad = [i for i, ob in zip(sub, obufs) if not np.array_equal(bufs[i], ob)]
    assert not bad, f"{len(bad)} of {len(sub)} sampled tiles differ, first {bad[:8]}"
    for i, orr in zip(sub, ores):
        assert (res[i].num_rays, res[i].num_queries) == (orr.num_rays, orr.num_queries)
    assert after.closest_queries > before.closest_queries


def test_c2_bench_schedule_full_frame(c2):
    """C2 as the bench renders it: the full 1920x1080 dragon stand-in frame (8 160 tiles, 2.07 M
    slots per pass, n_shadow = 1, kd stack class 48, not LDS-staged: three-kernel bounces) through
    render_split_pipelined with 4 units in flight in 2 task groups at 2 spp, the tail kernel taking
    over on the device once a pass holds fewer than 2^16 live paths (asserted: tail queries > 0).
    Every tile, ray and query count equals the same frame with sequential passes, and every 64th
    tile equals the oracle's (task.rs:25-82 pass order, renderer.rs:179-204 tasks)."""
    W, H, spp = 1920, 1080, 2
    cam = scenes.default_camera((W, H))
    tasks = L.make_tasks(W, H, spp, SEED)
    d = L.Device(0)
    try:
        d.upload(c2, cam)
        info = d.scene_info()
        assert info.n_shadow == 1 and info.stack_class == 48 and info.lds_bytes == 0 and info.top_kd_nodes > 0
        assert d.option("tail_below") == 1 << 16
        before = d.stats()
        bufs, res = d.render_tasks(tasks, max_paths=1 << 23)
        after = d.stats()
        sch = d.last_schedule()
        assert (sch.schedule, sch.units_in_flight, sch.task_groups, sch.fused) == (2, 4, 2, 0)
        assert after.tail_queries > before.tail_queries  # the mid-pass hand-over to the tail kernel ran
        d.set_option("split_pipe", 1)
        b2 = d.stats()
        seq, seq_res = d.render_tasks(tasks, max_paths=1 << 23)
        a2 = d.stats()
        assert d.last_schedule().schedule == 0
        # the same closest queries in all (where the tail kernel takes over differs: a task group's
        # unit holds half the frame's paths, so it drops below 2^16 live paths bounces earlier)
        assert a2.closest_queries - b2.closest_queries == after.closest_queries - before.closest_queries
    finally:
        d.close()
    for b, s, r, sr in zip(bufs, seq, res, seq_res):
        np.testing.assert_array_equal(b, s)
        assert (r.num_rays, r.num_queries) == (sr.num_rays, sr.num_queries)
    sub = list(range(0, len(tasks), 64))
    obufs, ores, _ = O.render_tasks(c2.desc(), cam.desc, [tasks[i] for i in sub], O.WAVEFRONT, oracle_threads())
    bad = [i for i, ob in zip(sub, obufs) if not np.array_equal(bufs[i], ob)]
    assert not bad, f"{len(bad)} of {len(sub)} sampled tiles differ, first {bad[:8]}"
    for i, orr in zip(sub, ores):
        assert (res[i].num_rays, res[i].num_queries) == (orr.num_rays, orr.num_queries)


@pytest.mark.parametrize("top_kb", [24, 64, 160])
def test_top_budget_caps_lds(top_kb):
    """LUMO_OPT_TOP_KB caps the TOP kernels' whole LDS use: the TOP set, the kd stack columns and
    the kd treelets together (top_shm) stay within the budget, and the tiles equal the oracle's."""
    sc = scenes.dragon(torus_knot_tube(300, 12)).build()
    d = L.Device(0, top_kb=top_kb)
    try:
        cam = scenes.default_camera((64, 48))
        d.upload(sc, cam)
        info = d.scene_info()
        assert 0 < info.top_shm <= top_kb * 1024
        tasks = L.make_tasks(64, 48, 4, SEED)[:6]
        bufs, res = d.render_tasks(tasks)
    finally:
        d.close()
    obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)


@pytest.mark.parametrize("top_kd,kd_lds", [(1, 8), (1, 4), (1, 0), (0, 8)])
def test_kd_treelets_in_lds(top_kd, kd_lds):
    """The TOP set's spare LDS holds the first treelets (top levels) of the largest kd tree
    (kdtree.rs:101-169 walked from LDS below the staged range, from HBM above it): on the small
    dragon (an instanced 7 200-triangle mesh, feature class 1) with 8 / 4 / 0 kd stack entries in
    LDS (more or less room for nodes) and with the staging off, lumo_trace (t / kind / object and
    traversal counters) and rendered tiles equal the oracle's."""
    sc = scenes.dragon(torus_knot_tube(300, 12)).build()
    d = L.Device(0, top_kd=top_kd, kd_lds=kd_lds)
    try:
        d.upload(sc)
        info = d.scene_info()
        assert info.lds_bytes == 0 and info.top_bytes > 0
        assert (info.top_kd_nodes > 0) == (top_kd == 1)
        desc = sc.desc()
        o, dd = _closest_rays(desc, (0.0, 0.0, 0.0), 1 << 16, 31)
        _trace_cmp(d, sc, o, dd)
        o, dd, li = _visibility_rays(desc, 1 << 16, 32)
        _trace_cmp(d, sc, o, dd, lights=li)
        cam = scenes.default_camera((64, 48))
        d.upload(sc, cam)
        tasks = L.make_tasks(64, 48, 4, SEED)[:8]
        bufs, res = d.render_tasks(tasks)
    finally:
        d.close()
    obufs, ores, _ = O.render_tasks(desc, cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
