"""GPU parity of the wide accel mode (LUMO_OPT_ACCEL = 1): the 4-wide SAH BVH the
upload builds (lumo_amd/csrc/common/wbvh_build.h) walked nearest child first by the HIP kernels
(dscene.h wide_walk) against the oracle's restatement of the same walk on the same structure
(oracle.cpp wide_walk).

Bar: BIT-EXACT, as for lumo's structures: every lumo_trace t / kind / object / triangle and the
traversal counters (child boxes tested, nodes visited, triangles tested), every path, tile, count
and BDPT splat.  How the wide mode's results relate to lumo's own structures (the same t except
where lumo's kd walk skips a hit, tests/test_wide.py) is a CPU test of the oracle."""
import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from lumo_amd import _ffi, scenes
from lumo_amd.procedural import torus_knot_tube
from parity import gpu_paths, oracle_threads
from scenes import default_camera, material_zoo
from test_gpu_scale import _closest_rays, _visibility_rays

pytestmark = pytest.mark.gpu
SEED = 0x1DE
BDPT = L.Integrator.BDPathTrace


@pytest.fixture(scope="module")
def dev():
    d = L.Device(0, accel=1)
    yield d
    d.close()


def _trace_cmp(dev, sc, o, d, lights=None):
    dev.upload(sc)
    assert dev.scene_info().accel == 1
    before = dev.stats()
    g = dev.trace(o, d, lights)
    after = dev.stats()
    t, kind, obj, prim, cnt = O.trace(sc.desc(), o, d, lights, accel=1, with_prim=True)
    np.testing.assert_array_equal(g[0], t)
    np.testing.assert_array_equal(g[1], kind)
    np.testing.assert_array_equal(g[2], obj)
    if lights is None:
        np.testing.assert_array_equal(g[3], prim)
    k = 0 if lights is None else 1
    got = [after.aabb_tests[k] - before.aabb_tests[k], after.kd_nodes[k] - before.kd_nodes[k],
           after.tri_tests[k] - before.tri_tests[k]]
    assert got == [cnt.aabb_tests, cnt.kd_nodes, cnt.tri_tests]
    return g


def _small_scenes():
    """name -> (scene maker, eye of the camera-like rays, camera maker)"""
    from test_instances_lights import light_scene, sphere_scene

    def look(o, t):
        return lambda res: L.Camera.builder().origin(*o).towards(*t).resolution(res).build()
    return {
        "cornell": (lambda: L.Scene.cornell_box(), (278.0, 273.0, -800.0), L.Camera.cornell_box),
        "zoo": (material_zoo, (0.0, 0.0, 0.0), default_camera),
        "caustics": (scenes.caustics, (0.0, 0.0, 2.0), scenes.caustics_camera),
        "small_dragon": (lambda: scenes.dragon(torus_knot_tube(300, 12)), (0.0, 0.0, 0.0), scenes.default_camera),
        "tri_lights": (lambda: light_scene("triangles"), (0.0, 0.5, 4.0), look((0.0, 0.5, 4.0), (0.0, -0.5, 0.0))),
        "instanced_rect": (lambda: light_scene("instanced_rect"), (0.0, 0.5, 4.0),
                           look((0.0, 0.5, 4.0), (0.0, -0.5, 0.0))),
        "spheres_env": (lambda: sphere_scene(env=True), (0.0, 0.3, 4.0), look((0.0, 0.3, 4.0), (0.0, 0.0, 0.0))),
    }


@pytest.mark.parametrize("name", ["cornell", "zoo", "caustics", "small_dragon", "tri_lights", "instanced_rect",
                                  "spheres_env"])
def test_wide_trace_small_scenes(dev, name):
    make, eye, _ = _small_scenes()[name]
    sc = make()
    sc.build()
    o, d = _closest_rays(sc.desc(), eye, 1 << 16, 5)
    g = _trace_cmp(dev, sc, o, d)
    assert np.mean(g[1] > 0) > 0.2
    o, d, li = _visibility_rays(sc.desc(), 1 << 16, 6)
    _trace_cmp(dev, sc, o, d, li)


@pytest.mark.parametrize("which", ["c2", "c3"])
def test_wide_trace_full_scale(dev, which):
    sc = scenes.dragon().build() if which == "c2" else scenes.bistro().build()
    eye = (0.0, 0.0, 0.0) if which == "c2" else (-16.0, 5.0, -1.0)
    o, d = _closest_rays(sc.desc(), eye, 1 << 20, 11)
    g = _trace_cmp(dev, sc, o, d)
    info = dev.scene_info()
    assert info.stack_class == 0 and info.wide_nodes > 1000 and info.top_wide_nodes > 0
    assert info.wide_stack <= 64
    assert np.mean(g[1] > 0) > 0.3
    o, d, li = _visibility_rays(sc.desc(), 1 << 20, 12)
    _trace_cmp(dev, sc, o, d, li)


def _paths(dev, sc, cam, task, integrator=0):
    dev.upload(sc, cam)
    assert dev.scene_info().accel == 1
    if integrator:
        _ffi.check(_ffi.load().lumo_debug_set_integrator(dev.ctx, integrator), "debug integrator")
    try:
        g = gpu_paths(dev, task)
    finally:
        _ffi.load().lumo_debug_set_integrator(dev.ctx, 0)
    o = O.trace_paths(sc.desc(), cam.desc, task, integrator=integrator, accel=1)
    for k in ("depth", "raster", "lam", "radiance", "delta"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)


@pytest.mark.parametrize("name", ["cornell", "zoo", "caustics", "small_dragon", "tri_lights", "instanced_rect",
                                  "spheres_env"])
@pytest.mark.parametrize("integrator", [0, BDPT], ids=["pt", "bdpt"])
def test_wide_paths(dev, name, integrator):
    make, _, camera = _small_scenes()[name]
    sc = make()
    sc.build()
    cam = camera((32, 32))
    _paths(dev, sc, cam, L.make_tasks(32, 32, 8, SEED)[1], integrator)


def _tiles_cmp(bufs, res, obufs, ores, sub=None, sp=None, osp=None):
    idx = sub if sub is not None else range(len(obufs))
    for k, i in enumerate(idx):
        np.testing.assert_array_equal(bufs[i], obufs[k])
        r, o = res[i], ores[k]
        assert (r.num_rays, r.num_queries, r.num_camera_rays) == (o.num_rays, o.num_queries, o.num_camera_rays)
        if sp is not None:
            assert len(sp[i]) == len(osp[k])
            np.testing.assert_array_equal(sp[i]["rgb"], osp[k]["rgb"])
            np.testing.assert_array_equal(sp[i]["x"], osp[k]["x"])


def test_wide_cornell_fused_tiles(dev):
    """Cornell with the wide trees staged whole in LDS: the fused bounce kernel (C1's path)."""
    sc = L.Scene.cornell_box()
    cam = L.Camera.cornell_box((64, 64))
    dev.upload(sc, cam)
    info = dev.scene_info()
    assert info.accel == 1 and info.lds_bytes > 0
    tasks = L.make_tasks(64, 64, 8, SEED)
    bufs, res = dev.render_tasks(tasks)
    assert dev.last_schedule().fused == 1
    obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, oracle_threads(), accel=1)
    _tiles_cmp(bufs, res, obufs, ores)


def test_wide_dragon_split_tiles(dev):
    """The small dragon through the split schedule (instanced mesh, TOP set of wide nodes)."""
    sc = scenes.dragon(torus_knot_tube(300, 12))
    cam = scenes.default_camera((48, 32))
    dev.upload(sc, cam)
    tasks = L.make_tasks(48, 32, 24, SEED)
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, oracle_threads(), accel=1)
    _tiles_cmp(bufs, res, obufs, ores)


def test_wide_bistro_standin_tiles(dev):
    """n_shadow > 1 (many triangle lights), the split pipeline with TOP kernels."""
    from lumo_amd.procedural import bistro_standin
    sc = scenes.bistro(bistro_standin(groups=40, lamps=64, n=4))
    cam = scenes.bistro_camera((48, 32))
    dev.upload(sc, cam)
    tasks = L.make_tasks(48, 32, 8, SEED)
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, oracle_threads(), accel=1)
    _tiles_cmp(bufs, res, obufs, ores)


@pytest.mark.parametrize("name,res,spp", [("cornell", (32, 32), 6), ("caustics", (40, 24), 4), ("zoo", (32, 16), 4)])
def test_wide_bdpt_tiles_and_splats(dev, name, res, spp):
    if name == "cornell":
        sc, cam = L.Scene.cornell_box(), L.Camera.cornell_box(res)
    elif name == "caustics":
        sc, cam = scenes.caustics(), scenes.caustics_camera(res)
    else:
        sc, cam = material_zoo(), default_camera(res)
    sc.build()
    dev.upload(sc, cam)
    tasks = L.make_tasks(res[0], res[1], spp, 0x5EED)
    sp, osp = [], []
    bufs, rr = dev.render_tasks(tasks, integrator=BDPT, splats_out=sp)
    obufs, orr, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8, integrator=BDPT, splats_out=osp,
                                   accel=1)
    assert sum(len(s) for s in osp) > 0
    _tiles_cmp(bufs, rr, obufs, orr, sp=sp, osp=osp)


def test_default_accel_is_lumo():
    d = L.Device(0)
    try:
        assert d.option("accel") == 0
        d.upload(L.Scene.cornell_box(), L.Camera.cornell_box((16, 16)))
        assert d.scene_info().accel == 0 and d.scene_info().stack_class == 4
    finally:
        d.close()


@pytest.mark.parametrize("mode", [1, 2])
def test_wide_ray_sort_matches_oracle(mode):
    """The counting sort (scan.h) of each bounce's closest-hit rays ahead of the wide walks: only
    the lane order changes, so the small dragon's tiles and counts equal the oracle's."""
    sc = scenes.dragon(torus_knot_tube(300, 12)).build()
    cam = scenes.default_camera((256, 192))
    d = L.Device(0, accel=1, ray_sort=mode, tail_below=0, split_groups=1)
    try:
        d.upload(sc, cam)
        tasks = L.make_tasks(256, 192, 2, SEED)
        bufs, res = d.render_tasks(tasks)
        assert d.stats().sorted_bounces > 0
    finally:
        d.close()
    obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, oracle_threads(), accel=1)
    _tiles_cmp(bufs, res, obufs, ores)


@pytest.mark.parametrize("n", [1, 2047, 2048, 2049, 5_000_001])
def test_device_exclusive_scan(n):
    """The hand-written exclusive scan (scan.h, two launches) that replaced the library scan of the
    BDPT item lists and splat taps, at sizes around its 2 048-count tile and across ~2 400 tiles."""
    import ctypes as C
    rng = np.random.default_rng(n)
    a = rng.integers(0, 40, size=n).astype(np.uint32)
    out = np.zeros(n, dtype=np.uint32)
    d = L.Device(0)
    try:
        _ffi.check(_ffi.load().lumo_debug_scan(d.ctx, a.ctypes.data_as(_ffi.c_uint32_p),
                                                out.ctypes.data_as(_ffi.c_uint32_p), C.c_size_t(n)), "debug_scan")
    finally:
        d.close()
    want = np.concatenate([[0], np.cumsum(a, dtype=np.uint64)[:-1]]).astype(np.uint32)
    np.testing.assert_array_equal(out, want)


def test_wide_lights_only_scene(dev):
    """A scene of lights only: the objects' tree is empty (root NONE), so every closest hit and
    visibility walk goes straight to the lights' tree; PT and BDPT tiles equal the oracle's."""
    from lumo_amd import Material, Spectrum
    sc = L.Scene()
    v, f = torus_knot_tube(100, 8)
    sc.add_mesh(v, f, Material.light(Spectrum.from_rgb(1.0, 0.8, 0.6), scale=0.5), light=True)
    sc.build()
    cam = L.Camera.builder().origin(0.0, 0.0, 3.0).towards(0.0, 0.0, 0.0).resolution((32, 32)).build()
    dev.upload(sc, cam)
    assert dev.scene_info().accel == 1
    assert O.wide_export(sc.desc())["obj_root"] == -(1 << 31)
    tasks = L.make_tasks(32, 32, 4, SEED)
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, oracle_threads(), accel=1)
    _tiles_cmp(bufs, res, obufs, ores)
    assert sum(float(b.sum()) for b in bufs) > 0.0
    sp, osp = [], []
    bufs, rr = dev.render_tasks(tasks, integrator=BDPT, splats_out=sp)
    obufs, orr, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8, integrator=BDPT, splats_out=osp,
                                   accel=1)
    _tiles_cmp(bufs, rr, obufs, orr, sp=sp, osp=osp)


def test_wide_texture_zoo(dev):
    """The texture feature class (image / procedural textures, bump map, textured light, HDR
    environment map) on the wide walks: PT tiles, BDPT tiles and splats equal the oracle's."""
    from scenes import texture_zoo
    zoo = texture_zoo().build()
    cam = default_camera((48, 32))
    dev.upload(zoo, cam)
    info = dev.scene_info()
    assert info.accel == 1 and info.full_kernels == 2
    tasks = L.make_tasks(48, 32, 8, SEED)
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(zoo.desc(), cam.desc, tasks, O.WAVEFRONT, oracle_threads(), accel=1)
    _tiles_cmp(bufs, res, obufs, ores)
    tasks = L.make_tasks(48, 32, 4, SEED)
    sp, osp = [], []
    bufs, rr = dev.render_tasks(tasks, integrator=BDPT, splats_out=sp)
    obufs, orr, _ = O.render_tasks(zoo.desc(), cam.desc, tasks, O.WAVEFRONT, 8, integrator=BDPT, splats_out=osp,
                                   accel=1)
    assert sum(len(s) for s in osp) > 0
    _tiles_cmp(bufs, rr, obufs, orr, sp=sp, osp=osp)
