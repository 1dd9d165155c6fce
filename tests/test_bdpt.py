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
