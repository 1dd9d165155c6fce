"""Procedural stand-ins for the reference's downloaded benchmark assets:
the assets (Stanford dragon, Amazon Bistro) are fetched from URLs by lumo's parser and are not
available offline, so the benchmark configurations use seeded procedural meshes with the same
triangle counts and the same scene structure."""
import numpy as np

DRAGON_TRIANGLES = 871_414  # dragon.obj as loaded by lumo


def torus_knot_tube(n_along, n_around, p=3, q=7, R=1.0, r_knot=0.42, r_tube=0.13, noise=0.02, seed=1):
    """Closed tube around a (p, q) torus knot: n_along x n_around quads -> 2 * n_along * n_around
    triangles, with seeded low-frequency radial noise so the surface is not trivially regular."""
    rng = np.random.default_rng(seed)
    t = np.arange(n_along) * (2 * np.pi / n_along)
    u = np.arange(n_around) * (2 * np.pi / n_around)

    def curve(tt):
        rr = R + r_knot * np.cos(q * tt)
        return np.stack([rr * np.cos(p * tt), r_knot * np.sin(q * tt), rr * np.sin(p * tt)], -1)

    c = curve(t)
    tang = curve(t + 1e-4) - curve(t - 1e-4)
    tang /= np.linalg.norm(tang, axis=1, keepdims=True)
    ref = np.array([0.0, 1.0, 0.0])
    n1 = np.cross(tang, ref)
    n1 /= np.linalg.norm(n1, axis=1, keepdims=True)
    n2 = np.cross(tang, n1)
    # seeded smooth radial modulation: a few random harmonics along and around the tube
    k = rng.integers(1, 40, size=(6, 2))
    ph = rng.uniform(0, 2 * np.pi, size=6)
    amp = rng.uniform(0.3, 1.0, size=6)
    T, U = np.meshgrid(t, u, indexing="ij")
    mod = sum(a * np.sin(kk[0] * T + kk[1] * U + f) for a, kk, f in zip(amp, k, ph)) / amp.sum()
    rad = r_tube * (1.0 + noise / r_tube * mod)
    v = (c[:, None, :] + rad[..., None] * (np.cos(U)[..., None] * n1[:, None, :] +
                                           np.sin(U)[..., None] * n2[:, None, :]))
    v = v.reshape(-1, 3)
    i = np.arange(n_along)[:, None]
    j = np.arange(n_around)[None, :]
    a = i * n_around + j
    b = ((i + 1) % n_along) * n_around + j
    c2 = ((i + 1) % n_along) * n_around + (j + 1) % n_around
    d = i * n_around + (j + 1) % n_around
    faces = np.stack([a, b, c2, d], -1).reshape(-1, 4)
    return v, faces


def dragon_standin(seed=1):
    """871 414-triangle closed mesh: (3, 7) torus-knot tube with 10 627 x 41 quads."""
    return torus_knot_tube(10627, 41, seed=seed)
