"""lumo's math-module tests restated over the oracle's helpers (whose vector algebra, common/vec.h,
is the device's; the device's spherical / complex / ONB code is held to the oracle bit for bit by
the GPU parity tests):

* math/spherical_utils/spherical_utils_tests.rs: same_hemisphere, cos/sin phi, cos2/sin2/sin
  theta and tan2 theta against the angle formulas at lumo's per-sample threshold
  EPSILON / sqrt(min(|z|, 1 - |z|)), tan2_theta infinite on the equator;
* tracer/onb.rs tests: both_directions (to_world(to_local(v)) == v within EPSILON);
* math/complex/complex_tests.rs: division by zero is NaN, a / a == 1 exactly, sqrt(0) has norm
  0, |norm(a) - norm_sqr(sqrt(a))| < EPSILON, (a - a) == 0;
* math/vec3/vec3_tests.rs: normalize() is_normalized (|len^2 - 1| < EPSILON) over random and
  1e10-scaled vectors;
* math/transform/transform_tests.rs `inv`: random chains of the Instanceable operations the
  builder composes (scale / translate / rotate x, y, z; the test's perspective factor is not an
  Instanceable operation) map points and directions back through the stored inverse.
Samples come from square_to_sphere of uniform squares (rng/maps.rs:49-55), as in the tests.
"""
import math

import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O

EPS = 1e-10  # lib.rs:67 (f64)
N = 100_000  # spherical_utils_tests.rs NUM_SAMPLES


def square_to_sphere(u):
    z = 1.0 - 2.0 * u[:, 1]
    r = np.sqrt(np.maximum(1.0 - z * z, 0.0))
    phi = 2.0 * np.pi * u[:, 0]
    return np.stack([r * np.cos(phi), r * np.sin(phi), z], 1)


@pytest.fixture(scope="module")
def dirs():
    return square_to_sphere(np.random.default_rng(42).random((N, 2)))


def test_spherical_functions(dirs):
    got = O.math(0, dirs)
    phi = np.arctan2(dirs[:, 1], dirs[:, 0])
    phi = np.where(phi < 0.0, phi + 2.0 * np.pi, phi)  # spherical_utils.rs:12-15
    theta = np.arccos(np.clip(dirs[:, 2], -1.0, 1.0))
    rlx = np.minimum(np.abs(dirs[:, 2]), 1.0 - np.abs(dirs[:, 2]))
    thr = EPS / np.sqrt(rlx)
    keep = thr < math.sqrt(EPS)  # the test's own precondition
    assert keep.mean() > 0.999
    refs = [np.cos(phi), np.sin(phi), np.cos(theta) ** 2, np.sin(theta) ** 2, np.sin(theta)]
    for k, ref in enumerate(refs):
        assert (np.abs(got[keep, k] - ref[keep]) < thr[keep]).all(), k
    ratio = got[keep, 5] / np.tan(theta[keep]) ** 2
    assert (np.abs(ratio - 1.0) < thr[keep]).all()


def test_tan2_theta_infinite():
    w = np.array([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [1.0, 1.0, -1.7976931348623157e308]])
    w[2] = O.math(3, w[2])[0, :3]  # Direction::new(1, 1, Float::MIN).normalize()
    assert np.isinf(O.math(0, w)[:, 5]).all()


def test_same_hemisphere(dirs):
    z, x, y = np.eye(3)[2], np.eye(3)[0], np.eye(3)[1]
    probes = np.array([np.r_[z, x + 0.1 * z], np.r_[z, -z], np.r_[y + 0.1 * z, -y + 0.1 * z]])
    assert list(O.math(4, probes)[:, 0]) == [1.0, 0.0, 1.0]
    wo, wi = dirs[: N // 2], dirs[N // 2:]
    a = O.math(4, np.c_[wo, wi])[:, 0]
    b = O.math(4, np.c_[wo, -wi])[:, 0]
    c = O.math(4, np.c_[-wo, -wi])[:, 0]
    ok = wo[:, 2] * wi[:, 2] != 0.0
    assert (a[ok] != b[ok]).all() and (a == c).all()


def test_onb_both_directions(dirs):
    w = np.array([1.23, 4.56, 7.89])
    v = np.array([9.87, 6.54, 3.21])
    w, v = w / np.linalg.norm(w), v / np.linalg.norm(v)
    back = O.math(1, np.r_[w, v])[0]
    assert np.linalg.norm(back - v) < EPS
    back = O.math(1, np.c_[dirs[: N // 2], dirs[N // 2:]])
    assert (np.linalg.norm(back - dirs[N // 2:], axis=1) < EPS).all()


def test_complex():
    a = (1.23, 4.56)
    r = O.math(2, np.array([[a[0], a[1], 0.0, 0.0]]))[0]
    assert np.isnan(r[0:6]).all()  # a / 0, a / 0.0, 1 / 0
    r = O.math(2, np.array([[a[0], a[1], a[0], a[1]]]))[0]
    assert (r[0], r[1]) == (1.0, 0.0)  # a / a
    assert (r[8], r[9]) == (0.0, 0.0)  # a - a
    norm_a = math.sqrt(a[0] ** 2 + a[1] ** 2)
    assert abs(norm_a - (r[6] ** 2 + r[7] ** 2)) < EPS  # |a| == |sqrt(a)|^2
    z = O.math(2, np.array([[0.0, 0.0, 1.0, 0.0]]))[0]
    assert math.sqrt(z[6] ** 2 + z[7] ** 2) == 0.0


def test_normalize_is_normalized():
    rng = np.random.default_rng(7)
    v = rng.random((10_000, 3))
    for x in (v, v * 1e10 * rng.random((10_000, 1))):
        assert (np.abs(O.math(3, x)[:, 3] - 1.0) < EPS).all()


def _mesh_transform(ops):
    s = L.Scene()
    s.add_rectangle([0, 5, 0], [1, 5, 0], [1, 5, 1], L.Material.light(L.Spectrum.from_rgb(1, 1, 1)), light=True)
    ref = s.add_mesh([[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 1, 2]], L.Material.lambertian(L.Spectrum.from_rgb(1, 1, 1)))
    for name, args in ops:
        getattr(ref, name)(*args)
    d = s.desc()
    t = d.transforms[0]
    return np.array(t.m[:]).reshape(4, 4), np.array(t.inv[:]).reshape(4, 4)


def test_transform_inverse_roundtrip():
    """transform_tests.rs `inv`: p -> M p -> M^-1 (M p) within EPSILON (distance squared), for
    points and directions, over random chains of 8 operations."""
    rng = np.random.default_rng(3)
    names = ["scale", "translate", "rotate_x", "rotate_y", "rotate_z"]
    for _ in range(60):
        ops = []
        for _ in range(8):
            k = rng.integers(0, 5)
            if k == 0:
                ops.append(("scale", tuple(rng.random(3) + 1e-3)))
            elif k == 1:
                ops.append(("translate", tuple(rng.random(3))))
            else:
                ops.append((names[k], (float(rng.random()),)))
        m, inv = _mesh_transform(ops)
        for _ in range(20):
            p = rng.random(3)
            h = m @ np.r_[p, 1.0]
            back = inv @ (h / h[3])
            assert np.sum((back[:3] / back[3] - p) ** 2) < EPS
            dd = inv[:3, :3] @ (m[:3, :3] @ p)
            assert np.sum((dd - p) ** 2) < EPS
