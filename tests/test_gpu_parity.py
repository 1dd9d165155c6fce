"""GPU parity: the HIP wavefront path vs the CPU oracle (wavefront sample order).

Bar: BIT-EXACT.  The kernels and the oracle share the deterministic transcendentals of
lumo_amd/csrc/common/lmath.h and compute in IEEE f64 without contraction, so every path's
radiance, wavelengths, raster position, depth, the adaptive-RR delta of every pass, and every
film tile are required to be identical to the last bit."""
import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from parity import gpu_paths, oracle_threads

pytestmark = pytest.mark.gpu

SEED = 0x5EED1234


@pytest.fixture(scope="module")
def dev():
    d = L.Device(0)
    yield d
    d.close()


@pytest.fixture(scope="module")
def cornell():
    return L.Scene.cornell_box()


def _cmp_paths(g, o):
    for k in ("depth", "raster", "lam", "radiance", "delta"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)


@pytest.mark.parametrize("res,spp,tile", [((32, 32), 4, 0), ((64, 48), 16, 5), ((40, 24), 9, 3)])
def test_paths_match_oracle(dev, cornell, res, spp, tile):
    cam = L.Camera.cornell_box(res)
    dev.upload(cornell, cam)
    tasks = L.make_tasks(res[0], res[1], spp, SEED)
    task = tasks[tile]
    _cmp_paths(gpu_paths(dev, task), O.trace_paths(cornell.desc(), cam.desc, task))


def test_tiles_match_oracle(dev, cornell):
    cam = L.Camera.cornell_box((64, 64))
    dev.upload(cornell, cam)
    tasks = L.make_tasks(64, 64, 8, SEED)
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert r.num_rays == orr.num_rays
        assert r.num_camera_rays == orr.num_camera_rays
        assert r.num_queries == orr.num_queries


def test_large_tiles_match_oracle(dev, cornell):
    """Tasks of more than 256 pixels (32x48 tiles) take the unfused finish + film kernels; lumo's
    16x16 tiles take the fused per-tile kernel.  Both are held to the oracle bit for bit."""
    from lumo_amd import _ffi
    cam = L.Camera.cornell_box((64, 48))
    dev.upload(cornell, cam)
    seeds = [t.seed for t in L.make_tasks(64, 48, 4, SEED)]
    tasks = (_ffi.TileTask * 2)(*[_ffi.TileTask((32 * i, 0), (32 * i + 32, 48), 0, 4, 4, seeds[i]) for i in range(2)])
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, 2)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        assert b.shape == (4 * 32 * 48,)
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)


def test_multi_batch_tiles_match_oracle(dev, cornell):
    """Two 256-spp batches + a ragged 44-spp batch (ring buffer wrap, RR delta in use) on a
    ragged frame (tiles clipped at the right/bottom edge)."""
    cam = L.Camera.cornell_box((40, 24))
    dev.upload(cornell, cam)
    tasks = L.make_tasks(40, 24, 300, SEED)
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, 16)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)


def test_wavefront_chunking_invariant(dev, cornell):
    """Size-independent property at a larger frame: results do not depend on how many paths
    are in flight (max_paths), and repeated renders are identical."""
    cam = L.Camera.cornell_box((256, 256))
    dev.upload(cornell, cam)
    tasks = L.make_tasks(256, 256, 64, SEED)
    a, ra = dev.render_tasks(tasks)
    b, rb = dev.render_tasks(tasks, max_paths=5000)
    c, _ = dev.render_tasks(tasks)
    for x, y, z in zip(a, b, c):
        np.testing.assert_array_equal(x, y)
        np.testing.assert_array_equal(x, z)
    assert sum(r.num_camera_rays for r in ra) == 256 * 256 * 64
    assert [r.num_rays for r in ra] == [r.num_rays for r in rb]


def test_renderer_api_matches_oracle(cornell):
    """Renderer(scene, camera).samples(n).seed(s).render() -> Film, as lumo's API."""
    cam = L.Camera.cornell_box((48, 32))
    film = L.Renderer(cornell, cam).samples(6).seed(99).render()
    tasks = L.make_tasks(48, 32, 6, 99)
    obufs, _, _ = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    ref = L.Film(48, 32)
    for t, b in zip(tasks, obufs):
        ref.add_tile(t, b)
    np.testing.assert_array_equal(film.pixels, ref.pixels)
    assert np.all(np.isfinite(film.rgb()))


def test_errors_are_loud(dev):
    with pytest.raises(Exception):
        L.Device(1 << 20)


@pytest.mark.parametrize("tm", [L.ToneMap.REINHARD, L.ToneMap.clamp(0.2)])
def test_tone_mapped_tiles_match_oracle(dev, cornell, tm):
    cam = L.Camera.cornell_box((32, 32))
    dev.upload(cornell, cam)
    tasks = L.make_tasks(32, 32, 8, SEED)
    bufs, _ = dev.render_tasks(tasks, tone_map=tm)
    obufs, _, _ = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, 8, tone_map=tm)
    for b, ob in zip(bufs, obufs):
        np.testing.assert_array_equal(b, ob)
    plain, _ = dev.render_tasks(tasks)
    assert not np.array_equal(np.concatenate(plain), np.concatenate(bufs))


def nan_normal_scene():
    """Cornell box + a glass (MfDielectric 0.03) quad whose shading normals are NaN: the BSDF pdf
    of a bounce off it is NaN.  path_trace.rs:47 breaks only on `p_scatter <= 0.0`, so a NaN pdf
    continues the path (one more bounce, a NaN throughput) in lumo and in the oracle."""
    sc = L.Scene.cornell_box()
    obj = (b"v 150 100 300\nv 400 100 300\nv 400 400 300\nv 150 400 300\n"
           b"vn 0 0 1\nvn 0 0 1\nvn 0 0 1\nvn 0 0 1\nf 1//1 2//2 3//3\nf 1//1 3//3 4//4\n")
    sc.add_obj(obj, L.Material.transparent(L.named_spectrum("MAGENTA"), 0.03, 1.5))
    sc.build()
    d = sc.desc()
    nrm = np.ctypeslib.as_array(d.normals, shape=(d.num_normals * 3,))
    nrm[:] = np.nan
    return sc


def test_nan_pdf_continues_path(dev):
    sc = nan_normal_scene()
    cam = L.Camera.cornell_box((32, 32))
    dev.upload(sc, cam)
    task = L.make_tasks(32, 32, 16, SEED)[1]
    g = gpu_paths(dev, task)
    o = O.trace_paths(sc.desc(), cam.desc, task)
    for k in ("depth", "raster", "lam", "radiance", "delta"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)
    assert np.isnan(g["radiance"]).any()  # the NaN pdf was reached (and counted, below)
    st = dev.stats()
    assert st.samples_nan > 0


@pytest.mark.parametrize("max_paths", [0, 3000])
def test_separate_result_buffers_match_oracle(dev, cornell, max_paths):
    """lumo_render_tiles with each task's rgb_w a separate allocation, in reverse address order
    and with gaps (how a C / Rust caller passes lumo's FilmTile buffers): the
    device's host-copy path (not the single-transfer path the Python wrapper's one allocation
    takes), alone and with the run split into chunks by max_paths."""
    import ctypes as C

    from lumo_amd import _ffi
    cam = L.Camera.cornell_box((48, 48))
    dev.upload(cornell, cam)
    tasks = L.make_tasks(48, 48, 8, SEED)
    n = len(tasks)
    arr = (_ffi.TileTask * n)(*tasks)
    res = (_ffi.TileResult * n)()
    bufs = [None] * n
    for i in reversed(range(n)):  # later tasks at lower addresses, padding between them
        t = tasks[i]
        P = (t.px_max[0] - t.px_min[0]) * (t.px_max[1] - t.px_min[1])
        bufs[i] = np.full(4 * P + 17, np.nan)
        res[i].rgb_w = bufs[i].ctypes.data_as(_ffi.c_double_p)
    cfg = _ffi.RenderCfg(0, 0, max_paths, 0, 0.0, 0, 0, None)
    _ffi.check(_ffi.load().lumo_render_tiles(dev.ctx, arr, n, C.byref(cfg), res), "render_tiles")
    obufs, ores, _ = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b[:len(ob)], ob)
        assert np.isnan(b[len(ob):]).all()  # nothing written past the tile
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)


@pytest.mark.parametrize("fused,tail,pipe", [(0, 0, 0), (0, 300, 0), (0, 1 << 30, 0), (0, 0, 1), (0, 300, 1),
                                             (1, 0, 0), (1, 300, 0),
                                             (1, 1 << 30, 0), (1, 0, 1), (-1, 1 << 18, 1), (-1, 1 << 18, 2), (-1, 1 << 18, 3)])
def test_bounce_modes_match_oracle(dev, cornell, fused, tail, pipe):
    """The three-kernel bounce and the fused bounce kernel (k_bounce_q: closest hit + shading +
    NEE pair in one launch), each without the tail kernel (tail 0), with the tail entered
    mid-pass (tail 300) and with every path run to its end in one launch (tail 2^30), and the
    pipelined passes (fused bounces on one or two head streams, tail / film / ring on another): paths,
    tiles and the closest / shadow query counts all equal the oracle's.  (Traversal counters are
    not compared here: the device answers p_sct == 0 records without traversal, the oracle
    traces them; lumo_trace's counter parity is in test_gpu_trace / test_gpu_scale.)"""
    dev.set_option("fused", fused).set_option("tail_below", tail).set_option("pipeline", pipe)
    try:
        cam = L.Camera.cornell_box((48, 40))
        dev.upload(cornell, cam)
        tasks = L.make_tasks(48, 40, 24, SEED)
        _cmp_paths(gpu_paths(dev, tasks[4]), O.trace_paths(cornell.desc(), cam.desc, tasks[4]))
        before = dev.stats()
        bufs, res = dev.render_tasks(tasks)
        after = dev.stats()
        obufs, ores, cnt = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
        for b, ob, r, orr in zip(bufs, obufs, res, ores):
            np.testing.assert_array_equal(b, ob)
            assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
        assert after.closest_queries - before.closest_queries == cnt.closest_queries
        assert after.shadow_queries - before.shadow_queries == cnt.shadow_queries
    finally:
        dev.set_option("fused", -1).set_option("tail_below", 1 << 16).set_option("pipeline", 3)


@pytest.mark.parametrize("dyn,grid", [(0, 384), (0, 7), (1, 2048), (1, 5)])
def test_fused_fetch_modes_match_oracle(dev, cornell, dyn, grid):
    """The fused bounce kernel's two ways of handing paths to blocks: static grid-stride stripes
    (dyn 0, the default, at the default grid of 1.5 blocks per CU and at a grid of 7 blocks, so
    every block strides many times) and blocks fetching 256 paths at a time from a counter
    (dyn 1).  Tiles, ray and query counts equal the oracle's."""
    d0, g0 = dev.option("dyn_fetch"), dev.option("lds_grid")
    assert (d0, g0) == (0, 384)
    dev.set_option("dyn_fetch", dyn).set_option("lds_grid", grid)
    try:
        cam = L.Camera.cornell_box((48, 40))
        dev.upload(cornell, cam)
        tasks = L.make_tasks(48, 40, 24, SEED)
        bufs, res = dev.render_tasks(tasks)
        obufs, ores, _ = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
        for b, ob, r, orr in zip(bufs, obufs, res, ores):
            np.testing.assert_array_equal(b, ob)
            assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
    finally:
        dev.set_option("dyn_fetch", d0).set_option("lds_grid", g0)


@pytest.mark.parametrize("heads", [4, 5, 6, 8])
def test_head_bounce_counts_match_oracle(cornell, heads):
    """Pipelined passes handing over to the tail kernel after 4, 5, 6 or 8 head bounces (the choice
    between the RR bounce on the head stream or in the tail kernel is a size heuristic; every
    count must give the oracle's tiles)."""
    d = L.Device(0, heads=heads, merge_passes=1)
    cam = L.Camera.cornell_box((48, 40))
    d.upload(cornell, cam)
    tasks = L.make_tasks(48, 40, 24, SEED)
    bufs, res = d.render_tasks(tasks)
    sch = d.last_schedule()
    d.close()
    assert (sch.schedule, sch.head_bounces, sch.merged_passes) == (1, heads, 1)
    obufs, ores, _ = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)


HEADLINE = (1536, 1536, 8)  # 2.36 M slots per pass >= 2^21: the automatic head count is 6, as at 1024^2


def test_headline_schedule_matches_oracle(cornell):
    """The exact schedule behind the C1 bench line, at a size where the device picks it by itself:
    a pass of >= 2^21 slots (6 head bounces, the RR bounce on the head stream), 3 head streams
    rotating 4 sets of queues / counters / per-slot outputs (8 passes: every set is reused),
    static grid-stride stripes, max_paths = 2^23 (bench.py --max-paths).  Every tile's pixels, ray and
    query counts, and the frame's closest / shadow query totals equal the oracle's (wavefront
    order).  Then the same frame without pipelining (pipeline 0: passes in sequence, one stream)
    must give the same bits: the cross-stream machinery adds nothing to any per-path result."""
    W, H, spp = HEADLINE
    d = L.Device(0)
    try:
        cam = L.Camera.cornell_box((W, H))
        d.upload(cornell, cam)
        assert d.scene_info().lds_bytes > 0  # the fused, LDS-staged kernels (C1's)
        tasks = L.make_tasks(W, H, spp, SEED)
        before = d.stats()
        bufs, res = d.render_tasks(tasks, max_paths=1 << 23)
        after = d.stats()
        # 6 fused head bounces and 2 more on the tail stream per pass, then the tail kernel
        assert after.launches[1] - before.launches[1] == (6 + 2) * spp
        sch = d.last_schedule()
        assert (sch.schedule, sch.head_streams, sch.head_bounces, sch.merged_passes, sch.tail_bounces) == (1, 3, 6, 1, 2)
        d.set_option("pipeline", 0)
        seq, seq_res = d.render_tasks(tasks, max_paths=1 << 23)
        assert d.last_schedule().schedule == 0
    finally:
        d.close()
    for b, s, r, sr in zip(bufs, seq, res, seq_res):
        np.testing.assert_array_equal(b, s)
        assert (r.num_rays, r.num_queries) == (sr.num_rays, sr.num_queries)
    obufs, ores, cnt = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, oracle_threads())
    bad = [i for i, (b, ob) in enumerate(zip(bufs, obufs)) if not np.array_equal(b, ob)]
    assert not bad, f"{len(bad)} of {len(tasks)} tiles differ, first {bad[:8]}"
    for r, orr in zip(res, ores):
        assert (r.num_rays, r.num_queries, r.num_camera_rays) == (orr.num_rays, orr.num_queries,
                                                                  orr.num_camera_rays)
    assert after.closest_queries - before.closest_queries == cnt.closest_queries
    assert after.shadow_queries - before.shadow_queries == cnt.shadow_queries


def dof_scene():
    """examples/dof.rs's layout without its downloaded teapots: the 20 x 20 floor at y = -1, the
    3 x 3 light rotated to face down at y = 8, and three spheres in a row along -z (the teapots'
    places) for the focus to fall on."""
    s = L.Scene()
    grey = L.Material.diffuse(L.Spectrum.from_srgb(200, 200, 200))
    s.add_rectangle((-10, -1, 10), (10, -1, 10), (10, -1, -10), grey)  # normal +y
    s.add_rectangle((-1.5, 8, -3.0), (1.5, 8, -3.0), (1.5, 8, 0.0), L.Material.light(L.named_spectrum("WHITE"),
                                                                                     scale=0.25), light=True)
    for i in range(3):
        s.add_sphere(0.25, L.Material.diffuse(L.Spectrum.from_srgb(255, 245, 255))).translate(0.0, -0.75, -1.0 * i)
    s.build()
    return s


def dof_camera(res, lens=0.03):
    """dof.rs:15-22: origin 0.75 (-X) + 0.25 Y, towards 0.75 (-Y) - Z, lens_radius(0.03),
    focal_length(|o - t|) (perspective: the orthographic variant is test_orthographic_*)."""
    o, t = np.array([-0.75, 0.25, 0.0]), np.array([0.0, -0.75, -1.0])
    return (L.Camera.builder().origin(*o).towards(*t).lens_radius(lens)
            .focal_length(float(np.linalg.norm(o - t))).resolution(res).build())


@pytest.mark.parametrize("which", ["cornell", "dof"])
def test_thin_lens_matches_oracle(dev, cornell, which):
    """Camera::add_dof (camera.rs:221-243) with lens_radius != 0: the lens sample (drawn for every
    camera ray, integrator.rs:56) moves the origin on the lens and aims at the focal plane.  Paths
    and tiles equal the oracle's, for the Cornell camera with an 8-unit lens focused at z = 280
    and for dof.rs's camera (lens 0.03, focal length |origin - towards|)."""
    res = (40, 32)
    if which == "cornell":
        scene, cam = cornell, L.Camera.cornell_box_builder().lens_radius(8.0).focal_length(1080.0).resolution(res).build()
    else:
        scene, cam = dof_scene(), dof_camera(res)
    assert cam.desc.lens_radius > 0
    dev.upload(scene, cam)
    tasks = L.make_tasks(res[0], res[1], 12, SEED)
    _cmp_paths(gpu_paths(dev, tasks[3]), O.trace_paths(scene.desc(), cam.desc, tasks[3]))
    bufs, res_ = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(scene.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res_, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
    # the lens matters: the same frame through a pinhole differs
    pin = dof_camera(res, 0.0) if which == "dof" else L.Camera.cornell_box(res)
    dev.upload(scene, pin)
    flat, _ = dev.render_tasks(tasks)
    assert not np.array_equal(np.concatenate(flat), np.concatenate(bufs))


def test_busy_time_is_a_union(dev, cornell):
    """lumo_stats_busy_ms: the union of the timed launches' intervals.  With pipelined passes
    (launches of one stage overlap on several streams) it is at most the sum of the launch
    durations and at most the render's wall time; a stage set's union is at least each member's."""
    import time
    from lumo_amd import _ffi
    lib = _ffi.load()
    cam = L.Camera.cornell_box((256, 256))
    dev.upload(cornell, cam)
    tasks = L.make_tasks(256, 256, 32, SEED)
    dev.set_option("timing", 1)
    try:
        lib.lumo_stats_reset(dev.ctx)
        t0 = time.perf_counter()
        dev.render_tasks(tasks)
        wall_ms = (time.perf_counter() - t0) * 1e3
        st = dev.stats()
        unit = dev.busy_ms([1, 4])
        allst = dev.busy_ms(range(len(_ffi.STAGES)))
    finally:
        dev.set_option("timing", 0)
    assert 0 < unit <= st.kernel_ms[1] + st.kernel_ms[4] + 1e-3
    assert max(dev.busy_ms([1]), dev.busy_ms([4])) <= unit + 1e-6
    assert unit <= allst <= wall_ms


@pytest.mark.parametrize("sampler", [L.SamplerType.Uniform, L.SamplerType.Jittered, L.SamplerType.Sobol,
                                     L.SamplerType.MultiJittered])
def test_samplers_match_oracle(dev, cornell, sampler):
    """Renderer::sampler (samplers.rs:6-17): every SamplerType's raster positions, paths and tiles
    equal the oracle's, over two 256-spp batches and a ragged one (300 spp: the batch offsets of
    Jittered / MultiJittered strata and Sobol's BATCH_STATES)."""
    cam = L.Camera.cornell_box((24, 16))
    dev.upload(cornell, cam)
    tasks = L.make_tasks(24, 16, 300, SEED)
    for t in (tasks[0], tasks[-1]):
        _cmp_paths(gpu_paths(dev, t, sampler), O.trace_paths(cornell.desc(), cam.desc, t, sampler=sampler))
    bufs, res = dev.render_tasks(tasks, sampler=sampler)
    obufs, ores, _ = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, oracle_threads(), sampler=sampler)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)


def test_sobol_length_limit(dev, cornell):
    """sobol_seq.rs SOBOL_MAX_LEN = 1023: lumo panics past it; the device refuses the call."""
    cam = L.Camera.cornell_box((16, 16))
    dev.upload(cornell, cam)
    with pytest.raises(Exception):
        dev.render_tasks(L.make_tasks(16, 16, 1024, SEED), sampler=L.SamplerType.Sobol)
    dev.render_tasks(L.make_tasks(16, 16, 1023, SEED)[:1], sampler=L.SamplerType.Sobol)


@pytest.mark.parametrize("lens", [0.0, 0.03])
def test_orthographic_matches_oracle(dev, lens):
    """CameraType::Orthographic (camera.rs:257-268): dof.rs's own camera (orthographic, lens 0.03,
    focal length |origin - towards|) and its pinhole variant: paths and tiles equal the oracle's."""
    from test_samplers import ortho_camera
    scene = dof_scene()
    cam = ortho_camera((40, 32), lens)
    dev.upload(scene, cam)
    tasks = L.make_tasks(40, 32, 12, SEED)
    _cmp_paths(gpu_paths(dev, tasks[2]), O.trace_paths(scene.desc(), cam.desc, tasks[2]))
    bufs, res_ = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(scene.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res_, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
    assert np.concatenate(bufs).sum() > 0


def test_orthographic_bdpt_refused(dev):
    from test_samplers import ortho_camera
    dev.upload(dof_scene(), ortho_camera((16, 16)))
    with pytest.raises(Exception):
        dev.render_tasks(L.make_tasks(16, 16, 1, SEED), integrator=L.Integrator.BDPathTrace, splats_out=[])


@pytest.mark.parametrize("merge,heads", [(1, 0), (2, 0), (3, 0), (8, 0), (0, 0), (4, 4), (3, 6)])
def test_merged_passes_match_oracle(cornell, merge, heads):
    """Merged passes of the fused pipeline (render_pipelined): M consecutive passes' cameras and
    head bounces run as one queue with virtual slots, their tails / films / rings pass by pass.
    24 passes with M = 1, 2, 3 (a ragged last unit), 8, automatic (0: the largest, 8, for this
    tiny frame) and with 4 or 6 head bounces (6 is cut to RR_DEPTH when M > 1): every path (per-pass
    delta included), tile, ray and query count equals the oracle's (task.rs:28-69 order)."""
    d = L.Device(0, merge_passes=merge, heads=heads)
    try:
        cam = L.Camera.cornell_box((48, 40))
        d.upload(cornell, cam)
        tasks = L.make_tasks(48, 40, 24, SEED)
        _cmp_paths(gpu_paths(d, tasks[4]), O.trace_paths(cornell.desc(), cam.desc, tasks[4]))
        before = d.stats()
        bufs, res = d.render_tasks(tasks)
        after = d.stats()
        sch = d.last_schedule()
    finally:
        d.close()
    m = merge if merge else 8
    want_heads = heads if heads else 5  # automatic: 5 for passes of < 2^21 slots
    assert (sch.schedule, sch.merged_passes, sch.head_bounces) == (1, m, min(want_heads, 5) if m > 1 else want_heads)
    obufs, ores, cnt = O.render_tasks(cornell.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
    assert after.closest_queries - before.closest_queries == cnt.closest_queries
    assert after.shadow_queries - before.shadow_queries == cnt.shadow_queries


def test_share_schedule_matches_sequential_and_oracle(cornell):
    """One rank's 1/8 share of the C1 frame (the tiles with index % 8 == 0 of 1024^2, 131 k slots
    per pass, bench.py --share) with the merged-pass schedule the device picks for it (8 passes per
    unit, 3 head streams): every tile, ray and query count equals the same share rendered with
    sequential passes on one stream, and every 8th tile of the share equals the oracle's."""
    from lumo_amd.dist import shard_tasks
    W = H = 1024
    spp = 24
    cam = L.Camera.cornell_box((W, H))
    tasks = shard_tasks(L.make_tasks(W, H, spp, SEED), W, H, 0, 8)
    d = L.Device(0)
    try:
        d.upload(cornell, cam)
        bufs, res = d.render_tasks(tasks)
        sch = d.last_schedule()
        d.set_option("pipeline", 0)
        seq, seq_res = d.render_tasks(tasks)
        assert d.last_schedule().schedule == 0
    finally:
        d.close()
    assert (sch.schedule, sch.head_streams, sch.merged_passes) == (1, 3, 8)
    for b, s, r, sr in zip(bufs, seq, res, seq_res):
        np.testing.assert_array_equal(b, s)
        assert (r.num_rays, r.num_queries) == (sr.num_rays, sr.num_queries)
    sub = list(range(0, len(tasks), 8))
    obufs, ores, _ = O.render_tasks(cornell.desc(), cam.desc, [tasks[i] for i in sub], O.WAVEFRONT, oracle_threads())
    for i, ob, orr in zip(sub, obufs, ores):
        np.testing.assert_array_equal(bufs[i], ob)
        assert (res[i].num_rays, res[i].num_queries) == (orr.num_rays, orr.num_queries)


def test_two_contexts_two_threads(cornell):
    """lumo's executors share nothing but the task receiver (pool.rs:17-38): two contexts on
    device 0, each driven from its own host thread with its own execution options (one pipelined
    with timing on, one with sequential passes), render disjoint tile sets concurrently, three
    times each; every tile equals one context's render of the whole frame, and each context keeps
    its own options and schedule (INTEGRATION.md's one-context-per-thread layout)."""
    import threading
    W = H = 256
    cam = L.Camera.cornell_box((W, H))
    tasks = list(L.make_tasks(W, H, 16, SEED))
    halves = [tasks[0::2], tasks[1::2]]
    ref = L.Device(0)
    ref.upload(cornell, cam)
    rbufs, rres = ref.render_tasks(tasks)
    ref.close()
    devs = [L.Device(0, timing=1), L.Device(0, pipeline=0, merge_passes=2)]
    for d in devs:
        d.upload(cornell, cam)
    out, errs = [None, None], []

    def run(k):
        try:
            for _ in range(3):
                out[k] = devs[k].render_tasks(halves[k])
        except Exception as e:  # noqa: BLE001 (re-raised below)
            errs.append(e)

    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    try:
        assert not errs, errs
        assert devs[0].option("timing") == 1 and devs[1].option("timing") == 0
        assert devs[0].last_schedule().schedule == 1 and devs[1].last_schedule().schedule == 0
        assert devs[0].stats().kernel_ms[1] > 0 and devs[1].stats().kernel_ms[1] == 0  # timing only in context 0
    finally:
        for d in devs:
            d.close()
    for k in range(2):
        bufs, res = out[k]
        for i, (b, r) in enumerate(zip(bufs, res)):
            np.testing.assert_array_equal(b, rbufs[2 * i + k])
            assert (r.num_rays, r.num_queries) == (rres[2 * i + k].num_rays, rres[2 * i + k].num_queries)


def test_option_api(dev):
    """lumo_set_option / lumo_get_option: per-context values, range checks (LUMO_ERR_INVALID)."""
    d2 = L.Device(0)
    try:
        dev.set_option("split_pipe", 2)
        assert dev.option("split_pipe") == 2 and d2.option("split_pipe") == 4
        for name, bad in (("bounce_threads", 96), ("split_pipe", 0), ("stack_class", 12), ("fused", 2),
                          ("merge_passes", 9), ("timing", 2)):
            with pytest.raises(RuntimeError, match="INVALID"):
                dev.set_option(name, bad)
        assert dev.option("poison") == 1  # the test session's LUMO_POISON (conftest)
        from lumo_amd import _ffi
        v = __import__("ctypes").c_int64()
        assert _ffi.load().lumo_get_option(dev.ctx, len(_ffi.OPTIONS), __import__("ctypes").byref(v)) == 1
    finally:
        dev.set_option("split_pipe", 4)
        d2.close()


@pytest.mark.gpu
def test_environment_overrides_warn():
    """Context creation reads the LUMO_* option overrides: a value that does not parse is ignored,
    an out-of-range one clamped, and a LUMO_* name that is no option (a misspelling such as
    LUMO_TAIL_BELOW for LUMO_TAIL) is reported, each with one line on stderr."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, LUMO_TAIL="abc", LUMO_MERGE="99", LUMO_TAIL_BELOW="5")
    code = ("import lumo_amd as L; d = L.Device(0); "
            "print(d.option('tail_below'), d.option('merge_passes')); d.close()")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == [str(1 << 16), "8"]
    assert "LUMO_TAIL=abc is not a number; ignored" in r.stderr
    assert "LUMO_MERGE=99 outside [0, 8]; using 8" in r.stderr
    assert "LUMO_TAIL_BELOW names no option; ignored" in r.stderr
