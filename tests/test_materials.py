"""Microfacet materials (microfacet.rs, bxdf/microfacet.rs) in the oracle: lumo's white-furnace
test (material/white_furnace_tests.rs), a sampling-vs-pdf histogram check in the spirit of
bxdf/sampling_tests.rs + chi2_tests.rs, pdf normalisation, and the delta / dispersion semantics."""
import math

import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from lumo_amd import named_spectrum as NS
from pyref import Xorshift


def one_material_scene(mat):
    s = L.Scene()
    idx = s._mat(mat)
    s.add_rectangle((-1e4, 1e4, -1e4), (-1e4 + 1, 1e4, -1e4), (-1e4 + 1, 1e4, -1e4 + 1),
                    L.Material.light(NS("WHITE")), light=True)
    return s, idx


MATERIALS = {
    "lambertian": lambda: L.Material.lambertian(NS("WHITE")),
    "diffuse": lambda: L.Material.diffuse(NS("WHITE")),
    "conductor75_eta15_k3": lambda: L.Material.metal(NS("WHITE"), 0.75, 1.5, 3.0),
    "conductor25_eta15_k3": lambda: L.Material.metal(NS("WHITE"), 0.25, 1.5, 3.0),
    "conductor00_eta15_k3": lambda: L.Material.metal(NS("WHITE"), 0.0, 1.5, 3.0),
    "conductor75_eta25_k0": lambda: L.Material.metal(NS("WHITE"), 0.75, 2.5, 0.0),
    "conductor10_eta25_k0": lambda: L.Material.metal(NS("WHITE"), 0.10, 2.5, 0.0),
    "dielectric75_eta15": lambda: L.Material.transparent(NS("WHITE"), 0.75, 1.5),
    "dielectric25_eta15": lambda: L.Material.transparent(NS("WHITE"), 0.25, 1.5),
    "dielectric00_eta15": lambda: L.Material.transparent(NS("WHITE"), 0.0, 1.5),
    "dielectric50_eta25": lambda: L.Material.transparent(NS("WHITE"), 0.50, 2.5),
    "dielectric10_eta25": lambda: L.Material.transparent(NS("WHITE"), 0.10, 2.5),
    "mirror": lambda: L.Material.mirror(),
    "glass": lambda: L.Material.glass(),
}


def square_to_hemisphere(u, v):
    z = u
    r = math.sqrt(max(0.0, 1.0 - z * z))
    phi = 2 * math.pi * v
    return np.array([r * math.cos(phi), r * math.sin(phi), z])


@pytest.mark.parametrize("name", sorted(MATERIALS))
def test_white_furnace(name):
    """white_furnace_tests.rs: no material returns more energy than it receives (< 1.01)."""
    s, m = one_material_scene(MATERIALS[name]())
    d = s.desc()
    rng = Xorshift(1234)
    for run in range(12):
        wo = square_to_hemisphere(*rng.gen_vec2())
        if wo[2] < 1e-3:
            continue
        r = O.furnace(d, m, wo, 16384, 77 + run)
        assert r.max() < 1.01, (name, wo, r)
        assert np.all(r >= 0.0)


ROUGH = ["diffuse", "conductor75_eta15_k3", "conductor25_eta15_k3", "conductor75_eta25_k0", "dielectric75_eta15",
         "dielectric25_eta15", "dielectric50_eta25", "lambertian"]


def _sphere_grid(nt, nphi):
    """midpoint grid uniform in (cos theta, phi) over the whole sphere; equal solid angle cells"""
    ct = -1 + (np.arange(nt) + 0.5) * 2.0 / nt
    ph = (np.arange(nphi) + 0.5) * 2 * np.pi / nphi
    C, P = np.meshgrid(ct, ph, indexing="ij")
    st = np.sqrt(1 - C * C)
    w = np.stack([st * np.cos(P), st * np.sin(P), C], -1).reshape(-1, 3)
    return w, 4 * np.pi / (nt * nphi)


@pytest.mark.parametrize("name", ROUGH)
def test_sampling_matches_pdf(name):
    """Histogram of bsdf_sample directions over 8x16 (cos theta, phi) bins of the sphere equals
    the pdf integrated over each bin (sampling_tests.rs / chi2_tests.rs)."""
    s, m = one_material_scene(MATERIALS[name]())
    d = s.desc()
    lam = np.array([550.0, 450.0, 650.0, 500.0])
    wo = np.array([0.3, -0.2, 0.0])
    wo[2] = math.sqrt(1 - wo[0] ** 2 - wo[1] ** 2)
    n = 400000
    wi, ok = O.bsdf_sample(d, m, wo, lam, n, 99)
    wi = wi[ok]
    nb_t, nb_p = 8, 16

    def bins(w):
        w = w / np.linalg.norm(w, axis=1, keepdims=True)
        bt = np.clip(((w[:, 2] + 1) / 2 * nb_t).astype(int), 0, nb_t - 1)
        bp = np.clip((np.mod(np.arctan2(w[:, 1], w[:, 0]), 2 * np.pi) / (2 * np.pi) * nb_p).astype(int), 0, nb_p - 1)
        return bt * nb_p + bp

    hist = np.bincount(bins(wi), minlength=nb_t * nb_p) / n
    grid, dw = _sphere_grid(8 * 40, 16 * 40)
    pdf, _ = O.bsdf_eval(d, m, wo, lam, grid)
    expect = np.bincount(bins(grid), weights=pdf * dw, minlength=nb_t * nb_p)
    assert np.abs(hist - expect).max() < 0.006, np.abs(hist - expect).max()
    # the pdf integrates to the probability that a sample is produced
    np.testing.assert_allclose(expect.sum(), ok.mean(), atol=0.01)


def test_delta_conductor_reflects_exactly():
    s, m = one_material_scene(L.Material.mirror())
    wo = np.array([0.3, 0.4, math.sqrt(1 - 0.25)])
    wi, ok = O.bsdf_sample(s.desc(), m, wo, np.array([550.0, 450.0, 650.0, 500.0]), 16, 5)
    assert ok.all()
    np.testing.assert_allclose(wi, np.tile([-0.3, -0.4, wo[2]], (16, 1)), atol=1e-15)


def test_dispersion_terminates_wavelengths():
    """Glass (eta 1.5 -> dispersive glass_eta) keeps only the hero wavelength after sampling;
    a constant-eta dielectric does not (bxdf/microfacet.rs:293-297, wavelength.rs:86-93)."""
    import ctypes as C
    from lumo_amd import _ffi
    s, m = one_material_scene(L.Material.transparent(NS("WHITE"), 0.0, 1.5))
    d = s.desc()
    mats = [d.materials[i] for i in range(d.num_materials)]
    assert (mats[m].flags & 1) == 0
    s2, m2 = one_material_scene(L.Material.transparent(NS("WHITE"), 0.0, 1.7))
    d2 = s2.desc()
    assert (d2.materials[m2].flags & 1) == 1
    # f of a refracted direction is evaluated with the terminated wavelengths in the path; the
    # eval hook takes lambda as given: zero wavelengths give zero Fresnel -> full transmission
    wo = np.array([0.0, 0.0, 1.0])
    pdf, f = O.bsdf_eval(d, m, wo, np.array([550.0, 0.0, 0.0, 0.0]), np.array([[0.0, 0.0, -1.0]]))
    assert f[0, 0] > 0 and np.all(f[0, 1:] == f[0, 1])
