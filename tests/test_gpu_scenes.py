"""GPU parity on scenes exercising instances, triangle lights and microfacet materials:
the examples/dragon.rs scene with a small procedural mesh, and a scene lit by emissive
triangles and an instanced, tilted rectangle light.  Bar: bit-exact per path and per tile."""
import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from lumo_amd import scenes
from lumo_amd.procedural import torus_knot_tube
from parity import gpu_paths
from test_instances_lights import light_scene

pytestmark = pytest.mark.gpu
SEED = 0xBEEF


@pytest.fixture(scope="module")
def dev():
    d = L.Device(0)
    yield d
    d.close()


def small_dragon():
    return scenes.dragon(torus_knot_tube(300, 12))


def _paths(dev, sc, cam, task):
    dev.upload(sc, cam)
    g = gpu_paths(dev, task)
    o = O.trace_paths(sc.desc(), cam.desc, task)
    for k in ("depth", "raster", "lam", "radiance", "delta"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)


@pytest.mark.parametrize("tile", [1, 6, 9])
def test_dragon_scene_paths(dev, tile):
    cam = scenes.default_camera((64, 48))
    _paths(dev, small_dragon(), cam, L.make_tasks(64, 48, 16, SEED)[tile])


@pytest.mark.parametrize("kind", ["triangles", "tilted_rect", "instanced_rect"])
def test_light_scene_paths(dev, kind):
    cam = L.Camera.builder().origin(0.0, 0.5, 4.0).towards(0.0, -0.5, 0.0).resolution((32, 32)).build()
    _paths(dev, light_scene(kind), cam, L.make_tasks(32, 32, 16, SEED)[2])


def test_dragon_scene_tiles(dev):
    sc = small_dragon()
    cam = scenes.default_camera((48, 32))
    dev.upload(sc, cam)
    tasks = L.make_tasks(48, 32, 24, SEED)
    bufs, res = dev.render_tasks(tasks)
    obufs, ores, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 16)
    for b, ob, r, orr in zip(bufs, obufs, res, ores):
        np.testing.assert_array_equal(b, ob)
        assert (r.num_rays, r.num_queries) == (orr.num_rays, orr.num_queries)


def test_trace_instanced(dev):
    sc = small_dragon()
    dev.upload(sc)
    rng = np.random.default_rng(3)
    o = rng.uniform([-0.9, -0.7, -1.9], [0.9, 0.7, -0.1], size=(50000, 3))
    d = rng.normal(size=(50000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    g = dev.trace(o, d)
    r = O.trace(sc.desc(), o, d)
    for a, b in zip(g[:3], r[:3]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("env", [False, True])
def test_sphere_scene_paths(dev, env):
    from test_instances_lights import sphere_scene
    cam = L.Camera.builder().origin(0.0, 0.3, 4.0).towards(0.0, 0.0, 0.0).resolution((32, 32)).build()
    _paths(dev, sphere_scene(env=env), cam, L.make_tasks(32, 32, 16, SEED)[1])


def test_bistro_standin_paths(dev):
    """Many Triangle lights (n_shadow = ilog2(#lights)), per-group meshes, metal + diffuse
    materials and the environment sphere."""
    from lumo_amd.procedural import bistro_standin
    sc = scenes.bistro(bistro_standin(groups=40, lamps=64, n=4))
    cam = scenes.bistro_camera((48, 32))
    _paths(dev, sc, cam, L.make_tasks(48, 32, 8, SEED)[4])


def test_obj_scene_paths(dev, tmp_path):
    from test_obj import MTL, OBJ
    (tmp_path / "s.obj").write_bytes(OBJ)
    (tmp_path / "s.mtl").write_bytes(MTL)
    sc = L.Scene.from_file(str(tmp_path / "s.obj"), mtllib=str(tmp_path / "s.mtl"))
    cam = L.Camera.builder().origin(0.0, 1.2, 4.0).towards(0.0, 0.5, 0.0).resolution((32, 32)).build()
    _paths(dev, sc, cam, L.make_tasks(32, 32, 16, SEED)[3])
