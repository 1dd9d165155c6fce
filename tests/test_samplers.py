"""Pixel samplers (samplers.rs: Uniform, Jittered, MultiJittered, Sobol) and the orthographic
camera (camera.rs:127-132, 257-268) on the CPU: the oracle's sampler points against an independent
pure-Python restatement (bit-exact), the strata each sampler promises, and the orthographic
camera description and rays.  The device runs the same code paths in test_gpu_parity.py."""
import math

import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from pyref import sampler_points

KINDS = [L.SamplerType.MultiJittered, L.SamplerType.Uniform, L.SamplerType.Jittered, L.SamplerType.Sobol]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("batch,total", [(0, 1), (0, 16), (0, 300), (1, 300), (3, 1023), (2, 1000), (0, 256)])
def test_sampler_points_match_restatement(kind, batch, total):
    for seed in (1, 0x5EED1234, 0xFFFFFFFFFFFFFFFF):
        got = O.sampler_points(kind, batch, total, seed)
        ref = np.array(sampler_points(kind, batch, total, seed))
        assert got.shape == (min(256, total - 256 * batch), 2)
        np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("kind", [L.SamplerType.Jittered, L.SamplerType.MultiJittered])
def test_stratified_samplers_cover_their_strata(kind):
    """Jittered / MultiJittered with a square sample count: one point per cell of the dim x dim
    grid (and, for MultiJittered, one per row and per column of the fine dim^2 grid)."""
    total = 256
    dim = 16
    pts = O.sampler_points(kind, 0, total, 77)
    assert np.all((pts >= 0) & (pts < 1))
    cells = {(int(x * dim), int(y * dim)) for x, y in pts}
    assert len(cells) == total
    if kind == L.SamplerType.MultiJittered:
        assert len({int(x * total) for x, _ in pts}) == total
        assert len({int(y * total) for _, y in pts}) == total


def test_sobol_is_a_shuffled_low_discrepancy_sequence():
    """SobolSampler: the XOR with the pixel seed (shuffle, samplers.rs:228-230) keeps the net
    property of the unshuffled points: 256 consecutive points from state 0 fall one per cell of a
    16 x 16 grid for seed 0, and the seed changes the points."""
    a = O.sampler_points(L.SamplerType.Sobol, 0, 1023, 0)
    grid = {(int(x * 16), int(y * 16)) for x, y in a}
    assert len(grid) >= 250
    b = O.sampler_points(L.SamplerType.Sobol, 0, 1023, 12345)
    assert not np.array_equal(a, b)


def test_sobol_beyond_its_length_is_rejected():
    with pytest.raises(AssertionError):
        O.sampler_points(L.SamplerType.Sobol, 0, 1024, 1)


def ortho_camera(res=(32, 24), lens=0.0):
    o, t = np.array([-0.75, 0.25, 0.0]), np.array([0.0, -0.75, -1.0])
    return (L.Camera.builder().origin(*o).towards(*t).camera_type(L.CameraType.Orthographic).lens_radius(lens)
            .focal_length(float(np.linalg.norm(o - t))).resolution(res).build())


def test_orthographic_camera_desc():
    """CameraBuilder::build with CameraType::Orthographic (builder.rs:145-170): camera_to_screen is
    orthographic_projection() = scale(1, 1, 1/(far - near)) * translation(0, 0, -near) with near 0,
    far 1, i.e. the identity; the desc is flagged orthographic."""
    cam = ortho_camera()
    assert cam.desc.orthographic == 1
    np.testing.assert_array_equal(np.array(cam.desc.camera_to_screen[0]), np.eye(4).ravel())
    np.testing.assert_array_equal(np.array(cam.desc.camera_to_screen[1]), np.eye(4).ravel())
    persp = L.Camera.builder().resolution((32, 24)).build()
    assert persp.desc.orthographic == 0


def test_orthographic_paths_render():
    """Camera::generate_ray for Orthographic (origin = raster_to_camera(raster), direction +z in
    camera space, then add_dof): the oracle renders dof.rs's camera, with and without its lens."""
    from test_gpu_parity import dof_scene
    sc = dof_scene()
    cam = ortho_camera((32, 24))
    task = L.make_tasks(32, 24, 4, 0x5EED1234)[0]
    p = O.trace_paths(sc.desc(), cam.desc, task)
    assert np.all(np.isfinite(p["radiance"]))
    assert p["radiance"].sum() > 0
    lens = O.trace_paths(sc.desc(), ortho_camera((32, 24), 0.03).desc, task)
    assert not np.array_equal(lens["radiance"], p["radiance"])


def test_orthographic_bdpt_is_unsupported():
    """camera.rs:348-351: Orthographic has no pdf_importance (unimplemented!()), so lumo's BDPT
    panics with it; the oracle (and the device) refuse the combination."""
    from test_gpu_parity import dof_scene
    sc = dof_scene()
    cam = ortho_camera()
    tasks = L.make_tasks(32, 24, 1, 1)[:1]
    with pytest.raises(AssertionError):
        O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 1, integrator=1, splats_out=[])
