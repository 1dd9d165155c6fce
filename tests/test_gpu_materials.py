"""GPU parity for the microfacet materials (MfDiffuse / MfConductor / MfDielectric incl.
dispersion): every path of the HIP wavefront path identical to the oracle's."""
import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from parity import gpu_paths
from scenes import default_camera, material_zoo

pytestmark = pytest.mark.gpu
SEED = 0xD1CE


@pytest.fixture(scope="module")
def dev():
    d = L.Device(0)
    yield d
    d.close()


@pytest.mark.parametrize("tile", [0, 7, 11])
def test_material_zoo_paths(dev, tile):
    sc = material_zoo()
    cam = default_camera((64, 48))
    dev.upload(sc, cam)
    task = L.make_tasks(64, 48, 16, SEED)[tile]
    g = gpu_paths(dev, task)
    o = O.trace_paths(sc.desc(), cam.desc, task)
    for k in ("depth", "raster", "lam", "radiance", "delta"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)


def test_material_zoo_tiles(dev):
    sc = material_zoo()
    cam = default_camera((64, 48))
    dev.upload(sc, cam)
    tasks = L.make_tasks(64, 48, 32, SEED)
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 16)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)
