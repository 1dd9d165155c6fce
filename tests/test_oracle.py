"""The CPU oracle (oracle/src/oracle.cpp, test infrastructure) against lumo's own property tests
and against the committed regression fixture tests/golden/cornell_oracle.npz."""
import math
import os

import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from pyref import Xorshift, mj_offsets
from test_host import CUBE_F, CUBE_V, tiny_light

GOLD = os.path.join(os.path.dirname(__file__), "golden", "cornell_oracle.npz")
INF = float("inf")


@pytest.fixture(scope="module")
def cornell32():
    sc = L.Scene.cornell_box()
    cam = L.Camera.cornell_box((32, 32))
    return sc, cam, L.make_tasks(32, 32, 8, 0x5EED1234)


def test_golden_fixture_reproduced(cornell32):
    """tools/gen_golden.py output: both sample orders, ray counts and a per-path dump."""
    g = np.load(GOLD)
    sc, cam, tasks = cornell32
    for mode, name in ((O.WAVEFRONT, "wavefront"), (O.LUMO_ORDER, "lumo_order")):
        bufs, res, _ = O.render_tasks(sc.desc(), cam.desc, tasks, mode, 2)
        np.testing.assert_array_equal(np.concatenate(bufs), g[name])
        np.testing.assert_array_equal(np.array([r.num_rays for r in res], dtype=np.uint64), g[name + "_rays"])
    p = O.trace_paths(sc.desc(), cam.desc, tasks[1])
    for k in ("radiance", "lam", "raster", "depth", "delta"):
        np.testing.assert_array_equal(p[k], g["paths_" + k])


def test_wavefront_raster_is_lumo_mj(cornell32):
    """Wavefront mode keeps lumo's camera-sample stream: pixel j of a task is seeded with the
    j-th gen_u64 of Xorshift::new(task.seed) (task.rs:36-39) and draws MultiJittered offsets
    (samplers.rs:135-193); checked against an independent Python restatement."""
    sc, cam, tasks = cornell32
    t = tasks[3]
    p = O.trace_paths(sc.desc(), cam.desc, t)
    W = t.px_max[0] - t.px_min[0]
    P = W * (t.px_max[1] - t.px_min[1])
    rng = Xorshift(t.seed)
    ras = p["raster"].reshape(t.samples, P, 2)
    for j in range(P):
        offs = mj_offsets(t.batch, t.total_samples, rng.gen_u64(), t.samples)
        want = np.array([(t.px_min[0] + j % W + ox, t.px_min[1] + j // W + oy) for ox, oy in offs])
        np.testing.assert_array_equal(ras[:, j, :], want)


def test_mj_stratification():
    """Correlated multi-jitter: one sample per coarse stratum and per fine row/column."""
    for seed in (1, 99, 12345):
        offs = np.array(mj_offsets(0, 16, seed, 16))
        assert np.all((offs >= 0) & (offs < 1))
        coarse = {(int(x * 4), int(y * 4)) for x, y in offs}
        assert len(coarse) == 16
        assert len({int(x * 16) for x, _ in offs}) == 16
        assert len({int(y * 16) for _, y in offs}) == 16


def test_sample_orders_agree_in_expectation():
    """lumo's tile-serial RNG order and the wavefront order are two estimators of the same image:
    the per-channel image means over 8 seeds each agree within 4 standard errors."""
    sc = L.Scene.cornell_box()
    cam = L.Camera.cornell_box((32, 32))
    runs = {}
    for mode in (O.WAVEFRONT, O.LUMO_ORDER):
        ms = []
        for seed in range(1, 9):
            tasks = L.make_tasks(32, 32, 32, seed)
            bufs, _, _ = O.render_tasks(sc.desc(), cam.desc, tasks, mode, 8)
            f = L.Film(32, 32)
            for t, b in zip(tasks, bufs):
                f.add_tile(t, b)
            ms.append(np.nanmean(f.rgb(), axis=(0, 1)))
        runs[mode] = np.array(ms)
    a, b = runs[O.WAVEFRONT], runs[O.LUMO_ORDER]
    se = np.sqrt(a.var(0, ddof=1) / len(a) + b.var(0, ddof=1) / len(b))
    z = np.abs(a.mean(0) - b.mean(0)) / se
    assert np.all(z < 4.0), z
    assert np.all(a.mean(0) > 0)


def test_libm_sensitivity_is_small(cornell32):
    """Building the oracle on glibc instead of lmath.h only flips rare ties: the path depths of
    >= 99% of the paths are unchanged."""
    if not os.path.exists(O.ORACLE_GLIBC_PATH):
        pytest.skip("glibc oracle variant not built")
    sc, cam, tasks = cornell32
    a = O.trace_paths(sc.desc(), cam.desc, tasks[1])
    b = O.trace_paths(sc.desc(), cam.desc, tasks[1], path=O.ORACLE_GLIBC_PATH)
    assert np.mean(a["depth"] == b["depth"]) >= 0.99
    np.testing.assert_array_equal(a["raster"], b["raster"])


# ---- geometry properties (kdtree_tests.rs, test_util.rs, scene_tests.rs) ---------------------

def unit_cube_scene():
    """kdtree_tests.rs 'cube' mesh scaled to unit size and centred (to_unit_size().to_origin(),
    applied to the vertices since instances are outside the implemented scope)."""
    v = np.array(CUBE_V, dtype=float)
    lo, hi = v.min(0), v.max(0)
    v = (v - (lo + hi) / 2) / (hi - lo).max()
    s = L.Scene()
    s.add_mesh(v, CUBE_F, L.Material.lambertian(L.Spectrum.from_rgb(0.5, 0.5, 0.5)))
    tiny_light(s)
    return s


def sphere_points(n, seed, radius):
    """5 * square_to_sphere(rng.gen_vec2()) (maps.rs) for uniformly spread ray origins."""
    rng = Xorshift(seed)
    out = []
    for _ in range(n):
        u, v = rng.gen_vec2()
        z = 1 - 2 * u
        r = math.sqrt(max(0.0, 1 - z * z))
        phi = 2 * math.pi * v
        out.append((radius * r * math.cos(phi), radius * r * math.sin(phi), radius * z))
    return np.array(out)


def test_kd_intersects_from_sphere():
    """kdtree_tests.rs:52-80: rays from a radius-5 sphere towards the origin all hit the mesh."""
    s = unit_cube_scene()
    xo = sphere_points(10000, 3, 5.0)
    # the cube mesh is open at the bottom (5 quads): skip rays that would enter through it
    keep = xo[:, 1] > -0.1
    xo = xo[keep]
    d = -xo / np.linalg.norm(xo, axis=1, keepdims=True)
    t, kind, obj, cnt = O.trace(s.desc(), xo, d)
    assert np.all(kind == 1) and np.all(obj == 0)
    assert np.all((t > 4.0) & (t < 5.0))
    assert cnt.closest_queries == len(xo)


def test_intersect_planar():
    """kdtree_tests.rs:25-49: a planar quad mesh is hit by a ray along its normal."""
    s = L.Scene()
    s.add_mesh(np.array([(-1, 0, 0), (1, 0, 0), (1, 1, 0), (-1, 1, 0)], dtype=float), [(0, 1, 2), (0, 2, 3)],
               L.Material.lambertian(L.Spectrum.from_rgb(0.5, 0.5, 0.5)))
    tiny_light(s)
    t, kind, _, _ = O.trace(s.desc(), np.array([(0.0, 0.5, 0.5)]), np.array([(0.0, 0.0, -1.0)]))
    assert kind[0] == 1 and t[0] == pytest.approx(0.5, abs=1e-12)


def test_object_misses():
    """test_util.rs:3-24 analogues on the unit cube: a ray pointing away and a grazing ray just
    outside the boundary miss."""
    s = unit_cube_scene()
    o = np.array([(2.0, 0.0, 0.0), (0.5 + 1e-10 + 1e-3, 0.0, 0.0)])
    d = np.array([(1.0, 0.0, 0.0), (0.0, 0.0, 1.0)])
    t, kind, _, _ = O.trace(s.desc(), o, d)
    assert np.all(kind == 0) and np.all(np.isinf(t))


def disk_scene(with_blocker=True):
    """scene_tests.rs:6-25: a small light above a large occluding plate at y = 1 (disks replaced
    by rectangles; spheres and disks are outside the implemented scope)."""
    s = L.Scene()
    white = L.Spectrum.from_rgb(1.0, 1.0, 1.0)
    e = 1e-3
    s.add_rectangle((-e, 2.0, -e), (e, 2.0, -e), (e, 2.0, e), L.Material.light(white, two_sided=True), light=True)
    if with_blocker:
        s.add_rectangle((-100.0, 1.0, -100.0), (100.0, 1.0, -100.0), (100.0, 1.0, 100.0),
                        L.Material.lambertian(L.Spectrum.from_rgb(0.5, 0.5, 0.5)))
    return s


def test_light_no_pass():
    """scene_tests.rs:27-35: the light is not visible through the plate."""
    t, kind, _, _ = O.trace(disk_scene().desc(), np.array([(0.0, 0.0, 0.0)]), np.array([(0.0, 1.0, 0.0)]),
                            lights=np.array([0]))
    assert kind[0] == 0 and np.isinf(t[0])


def test_object_behind_light():
    """scene_tests.rs:37-45: a ray from above the light reaches it; the plate behind is ignored."""
    t, kind, obj, _ = O.trace(disk_scene().desc(), np.array([(0.0, 3.0, 0.0)]), np.array([(0.0, -1.0, 0.0)]),
                              lights=np.array([0]))
    assert kind[0] == 2 and obj[0] == 0 and t[0] == pytest.approx(1.0)
    # without the plate the light is visible from below as well
    t, kind, _, _ = O.trace(disk_scene(False).desc(), np.array([(0.0, 0.0, 0.0)]), np.array([(0.0, 1.0, 0.0)]),
                            lights=np.array([0]))
    assert kind[0] == 2 and t[0] == pytest.approx(2.0)


def test_hits_closest():
    """scene_tests.rs:47-75: the nearer of two parallel plates is reported."""
    s = L.Scene()
    grey = L.Material.lambertian(L.Spectrum.from_rgb(0.5, 0.5, 0.5))
    s.add_rectangle((-100.0, 2.0, -100.0), (100.0, 2.0, -100.0), (100.0, 2.0, 100.0), grey)
    s.add_rectangle((-100.0, 1.0, -100.0), (100.0, 1.0, -100.0), (100.0, 1.0, 100.0), grey)
    s.add_rectangle((-1.0, -100.0, -1.0), (1.0, -100.0, -1.0), (1.0, -100.0, 1.0),
                    L.Material.light(L.Spectrum.from_rgb(1.0, 1.0, 1.0)), light=True)
    t, kind, obj, _ = O.trace(s.desc(), np.array([(0.0, 0.0, 0.0)]), np.array([(0.0, 1.0, 0.0)]))
    assert kind[0] == 1 and t[0] == pytest.approx(1.0)
    t, kind, _, _ = O.trace(s.desc(), np.array([(0.0, 0.0, 0.0)]), np.array([(0.0, -1.0, 0.0)]))
    assert kind[0] == 2 and t[0] == pytest.approx(100.0)


def test_cornell_counters_consistent(cornell32):
    sc, cam, tasks = cornell32
    _, res, cnt = O.render_tasks(sc.desc(), cam.desc, tasks[:2], O.WAVEFRONT, 1)
    cams = sum(r.num_camera_rays for r in res)
    assert cams == 2 * 16 * 16 * 8
    assert sum(r.num_queries for r in res) == cnt.closest_queries + cnt.shadow_queries
    assert cnt.closest_queries >= cams
