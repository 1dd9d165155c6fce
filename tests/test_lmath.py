"""The render path's deterministic transcendentals (lumo_amd/csrc/common/lmath.h) stay within
2 ulp of the platform libm over the ranges the path evaluates them on."""
import ctypes as C
import math

import numpy as np
import pytest

import lumo_amd as L
from lumo_amd import _ffi

CASES = [(0, np.exp, -12.0, 3.0), (1, np.log1p, -0.99, 13.0), (2, np.cosh, -1.5, 2.5), (3, np.sin, -0.8, 7.0),
         (4, np.cos, -0.8, 7.0), (5, np.arctan, -30.0, 30.0), (6, np.arccos, -1.0, 1.0)]


@pytest.mark.parametrize("which,ref,lo,hi", CASES)
def test_lmath_close_to_libm(which, ref, lo, hi):
    x = np.random.default_rng(which).uniform(lo, hi, 200000)
    y = np.zeros_like(x)
    L.lib().lumo_lmath(which, x.ctypes.data_as(_ffi.c_double_p), y.ctypes.data_as(_ffi.c_double_p), len(x))
    r = ref(x)
    ulp = np.spacing(np.abs(r))
    err = np.abs(y - r) / ulp
    assert err.max() <= 2.0, err.max()
    assert np.mean(y == r) > 0.75  # most results are the correctly-rounded value


def test_lmath_special_values():
    x = np.array([0.0, -0.0, 1e-300, -1e-300, 700.0, -700.0, 1e-9])
    y = np.zeros_like(x)
    L.lib().lumo_lmath(0, x.ctypes.data_as(_ffi.c_double_p), y.ctypes.data_as(_ffi.c_double_p), len(x))
    assert y[0] == 1.0 and y[1] == 1.0
    np.testing.assert_allclose(y[4], math.exp(700.0), rtol=1e-15)
    np.testing.assert_allclose(y[5], math.exp(-700.0), rtol=1e-15)


def test_atan2_quadrants():
    """lm_atan2 (via the oracle's Complex::sqrt path) is exercised on the device; here the host
    atan (which=5) plus the identity atan2(y, x) = atan(y / x) + quadrant offsets are spot-checked
    against numpy at the axes and diagonals."""
    x = np.array([-1e300, -2.0, -1.0, -1e-300, 0.0, 1e-300, 1.0, 2.0, 1e300, np.inf, -np.inf])
    y = np.zeros_like(x)
    L.lib().lumo_lmath(5, x.ctypes.data_as(_ffi.c_double_p), y.ctypes.data_as(_ffi.c_double_p), len(x))
    np.testing.assert_allclose(y, np.arctan(x), rtol=2.3e-16, atol=0)


def _lm(which, x):
    y = np.zeros_like(x)
    L.lib().lumo_lmath(which, x.ctypes.data_as(_ffi.c_double_p), y.ctypes.data_as(_ffi.c_double_p), len(x))
    return y


def test_sincos_same_bits_as_sin_and_cos():
    """lm_sincos (the disk and sphere maps, rng.h) returns exactly lm_sin's and lm_cos's values: the
    arguments of square_to_disk (|theta| <= 3 pi / 4 and the pi / 4 boundaries), of
    square_to_sphere (0 .. 2 pi), multiples of pi / 4 around the reduction's branch points, large
    and tiny arguments, both signs, and NaN / inf."""
    rng = np.random.default_rng(7)
    q = np.pi / 4
    x = np.concatenate([rng.uniform(-3 * q, 3 * q, 100000), rng.uniform(0.0, 2 * np.pi, 100000),
                        rng.uniform(-1e5, 1e5, 20000),
                        np.array([k * q for k in range(-16, 17)]),
                        np.nextafter(np.array([k * q for k in range(-16, 17)]), np.inf),
                        np.nextafter(np.array([k * q for k in range(-16, 17)]), -np.inf),
                        np.array([0.0, -0.0, 1e-300, -1e-300, 1e-9, 3e5, -3e5, np.nan, np.inf, -np.inf])])
    s, c = _lm(7, x), _lm(8, x)
    np.testing.assert_array_equal(s.view(np.uint64), _lm(3, x).view(np.uint64))
    np.testing.assert_array_equal(c.view(np.uint64), _lm(4, x).view(np.uint64))
