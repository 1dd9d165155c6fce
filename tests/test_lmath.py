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
