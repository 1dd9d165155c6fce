"""GPU parity: the HIP wavefront path vs the CPU oracle (wavefront sample order).

Bar: BIT-EXACT.  The kernels and the oracle share the deterministic transcendentals of
lumo_amd/csrc/common/lmath.h and compute in IEEE f64 without contraction, so every path's
radiance, wavelengths, raster position, depth, the adaptive-RR delta of every pass, and every
film tile are required to be identical to the last bit."""
import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from parity import gpu_paths

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
