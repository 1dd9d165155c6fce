"""BDPT (integrator/bd_path_trace*.rs) in the oracle.  lumo's MIS test checks that the weights of
all strategies of a path sum to one; here the equivalent integral property is pinned: BDPT
(camera paths + light paths + all connections, MIS weighted, with light-tracing splats) and
PathTrace estimate the same image, so their image means agree within a few standard errors.
Wrong MIS weights or a missing strategy show up as a bias."""
import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from scenes import default_camera, material_zoo


def _means(scene, cam, res, spp, seeds, integrator):
    out = []
    for seed in seeds:
        tasks = L.make_tasks(res[0], res[1], spp, seed)
        sp = []
        bufs, _, _ = O.render_tasks(scene.desc(), cam.desc, tasks, O.WAVEFRONT, 8, integrator=integrator,
                                    splats_out=sp)
        f = L.Film(res[0], res[1], samples=spp)
        for t, b, s in zip(tasks, bufs, sp):
            f.add_tile(t, b, s)
        out.append(np.nanmean(f.rgb(), axis=(0, 1)))
    return np.array(out)


@pytest.mark.parametrize("which", ["cornell", "zoo"])
def test_bdpt_matches_path_trace_in_expectation(which):
    if which == "cornell":
        sc, cam, res = L.Scene.cornell_box(), L.Camera.cornell_box((24, 24)), (24, 24)
    else:
        sc, res = material_zoo(), (24, 16)
        cam = default_camera(res)
    seeds = range(1, 7)
    a = _means(sc, cam, res, 24, seeds, 0)
    b = _means(sc, cam, res, 24, [s + 100 for s in seeds], 1)
    se = np.sqrt(a.var(0, ddof=1) / len(a) + b.var(0, ddof=1) / len(b))
    z = np.abs(a.mean(0) - b.mean(0)) / se
    assert np.all(z < 4.0), (a.mean(0), b.mean(0), z)


def test_bdpt_splats_and_counters():
    sc, cam = L.Scene.cornell_box(), L.Camera.cornell_box((16, 16))
    tasks = L.make_tasks(16, 16, 4, 9)
    sp = []
    bufs, res, cnt = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 4, integrator=1, splats_out=sp)
    n = sum(len(s) for s in sp)
    assert n > 0
    for s in sp:
        assert np.all(s["x"] < 16) and np.all(s["y"] < 16) and np.isfinite(s["rgb"]).all()
    # cost counts vertices + connections: well above the path tracer's depth
    _, res_pt, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 4)
    assert sum(r.num_rays for r in res) > 2 * sum(r.num_rays for r in res_pt)
    # deterministic
    sp2 = []
    bufs2, _, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 4, integrator=1, splats_out=sp2)
    for x, y in zip(bufs, bufs2):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(sp, sp2):
        np.testing.assert_array_equal(x, y)


def _mis_scene(kind):
    """The scenes of bd_path_trace/mis_tests.rs:9-94 (the orthographic camera and the medium
    variants are out of scope here)."""
    if kind == "big_scale":
        cam = L.Camera.builder().origin(278.0, 273.0, -800.0).towards(278.0, 273.0, 0.0).zoom(2.8) \
            .focal_length(0.035).resolution((512, 512)).build()
        return L.Scene.cornell_box(), cam
    sc = L.Scene.empty_box(L.named_spectrum("WHITE"), L.Material.diffuse(L.named_spectrum("RED")),
                           L.Material.lambertian(L.named_spectrum("GREEN")))
    white = L.named_spectrum("WHITE")
    if kind == "specular_delta":
        sc.add_sphere(0.25, L.Material.mirror()).translate(-0.45, -0.5, -1.5)
        sc.add_sphere(0.25, L.Material.glass()).translate(0.45, -0.5, -1.3)
    elif kind == "specular_rough":
        sc.add_sphere(0.25, L.Material.metal(white, 0.5, 1.5, 1.5)).translate(-0.45, -0.5, -1.5)
        sc.add_sphere(0.25, L.Material.transparent(white, 0.5, 1.5)).translate(0.45, -0.5, -1.3)
    return sc, L.Camera.builder().build()


@pytest.mark.parametrize("kind", ["diffuse", "specular_delta", "specular_rough", "big_scale"])
def test_mis_weights_sum_to_one(kind):
    """mis_tests.rs all_sum_to_one_*: for full paths built from the light and from the camera,
    the MIS weights of every strategy the integrator evaluates sum to 1 (|1 - sum| < 0.01, lumo's
    bound), here for 10 000 paths per scene on the oracle's restated mis::weight."""
    sc, cam = _mis_scene(kind)
    sums, lens = O.mis_sums(sc.build().desc(), cam.desc, 10_000, 0x5EED + len(kind))
    assert np.all(np.abs(1.0 - sums) < 0.01), (kind, sums[np.abs(1.0 - sums) >= 0.01][:5])
    assert lens.min() >= 3 and lens.max() > 4  # paths of several lengths were exercised
