"""GPU parity of textures (texture.rs:53-92, image.rs:99-184, perlin.rs) and bump maps
(material.rs:323-331): every path, tile and BDPT splat of the HIP kernels over the texture zoo
(checkerboard of marble / Mandelbrot, PNG images incl. a packed palette, image ks and tf, bump
map, textured light, HDR environment map) identical to the oracle, plus a zipped OBJ scene with
map_Kd / map_Bump / map_Ke statements."""
import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from lumo_amd import _ffi
from parity import gpu_paths
from scenes import default_camera, texture_zoo, textured_obj_zip

pytestmark = pytest.mark.gpu
SEED = 0x7E47
BDPT = L.Integrator.BDPathTrace


@pytest.fixture(scope="module")
def dev():
    d = L.Device(0)
    yield d
    d.close()


@pytest.fixture(scope="module")
def zoo():
    return texture_zoo().build()


def _cmp(g, o):
    for k in ("depth", "raster", "lam", "radiance", "delta"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)


@pytest.mark.parametrize("tile", [0, 5, 9, 11])
def test_texture_zoo_paths(dev, zoo, tile):
    cam = default_camera((64, 48))
    dev.upload(zoo, cam)
    assert dev.scene_info().full_kernels == 2  # the texture feature class
    task = L.make_tasks(64, 48, 16, SEED)[tile]
    _cmp(gpu_paths(dev, task), O.trace_paths(zoo.desc(), cam.desc, task))


def test_texture_zoo_tiles(dev, zoo):
    cam = default_camera((64, 48))
    dev.upload(zoo, cam)
    tasks = L.make_tasks(64, 48, 16, SEED)
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(zoo.desc(), cam.desc, tasks, O.WAVEFRONT, 16)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)


@pytest.mark.parametrize("tile", [0, 3])
def test_texture_zoo_bdpt_paths(dev, zoo, tile):
    cam = default_camera((32, 32))
    dev.upload(zoo, cam)
    task = L.make_tasks(32, 32, 8, SEED)[tile]
    _ffi.check(_ffi.load().lumo_debug_set_integrator(dev.ctx, BDPT), "debug integrator")
    try:
        g = gpu_paths(dev, task)
    finally:
        _ffi.load().lumo_debug_set_integrator(dev.ctx, 0)
    _cmp(g, O.trace_paths(zoo.desc(), cam.desc, task, integrator=BDPT))


def test_texture_zoo_bdpt_tiles_and_splats(dev, zoo):
    cam = default_camera((32, 24))
    dev.upload(zoo, cam)
    tasks = L.make_tasks(32, 24, 4, SEED)
    sp, osp = [], []
    bufs, rr = dev.render_tasks(tasks, integrator=BDPT, splats_out=sp)
    obufs, orr, _ = O.render_tasks(zoo.desc(), cam.desc, tasks, O.WAVEFRONT, 8, integrator=BDPT, splats_out=osp)
    assert sum(len(s) for s in osp) > 0
    for b, ob, r, o, s, os_ in zip(bufs, obufs, rr, orr, sp, osp):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (o.num_rays, o.num_queries)
        for k in ("x", "y", "rgb"):
            np.testing.assert_array_equal(s[k], os_[k])


def test_textured_obj_scene(dev, tmp_path):
    """parser::scene_from_file of a zip whose MTL uses map_Kd / map_Bump / map_Ke."""
    p = textured_obj_zip(tmp_path / "scene.zip")
    sc = L.Scene.from_file(str(p), "scene.obj").build()
    cam = default_camera((32, 32))
    dev.upload(sc, cam)
    assert dev.scene_info().full_kernels == 2  # the texture feature class
    tasks = L.make_tasks(32, 32, 8, SEED)
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
    for b, ob in zip(bufs, obufs):
        np.testing.assert_array_equal(b, ob)
    assert sum(float(b.reshape(-1, 4)[:, :3].sum()) for b in bufs) > 0.0
