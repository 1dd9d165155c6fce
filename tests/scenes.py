"""Small test scenes built through lumo_amd's builder API (shared by CPU and GPU tests)."""
import numpy as np

import lumo_amd as L
from lumo_amd import named_spectrum as NS


def cube_mesh(center, size, rot_y=0.0):
    """Axis-aligned cube (optionally rotated about y) as 6 quads with outward winding."""
    h = size / 2.0
    v = np.array([[x, y, z] for x in (-h, h) for y in (-h, h) for z in (-h, h)], dtype=float)
    c, s = np.cos(rot_y), np.sin(rot_y)
    R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    v = v @ R.T + np.asarray(center, dtype=float)
    # vertex index = 4*ix + 2*iy + iz
    faces = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    return v, faces


def material_zoo():
    """empty_box (dragon.rs colours) with one cube per microfacet material kind."""
    s = L.Scene.empty_box(L.Spectrum.from_srgb(242, 242, 242), L.Material.diffuse(NS("RED")),
                          L.Material.diffuse(NS("GREEN")))
    mats = [L.Material.metal(L.Spectrum.from_srgb(230, 180, 90), 0.3, 1.5, 3.0),
            L.Material.mirror(),
            L.Material.glass(),
            L.Material.transparent(NS("MAGENTA"), 0.03, 1.5),
            L.Material.transparent(NS("CYAN"), 0.2, 1.7),
            L.Material.lambertian(L.Spectrum.from_rgb(0.3, 0.5, 0.7))]
    pos = [(-0.6, -0.55, -1.5), (0.0, -0.55, -1.6), (0.6, -0.55, -1.5), (-0.45, -0.55, -0.9), (0.45, -0.55, -0.9),
           (0.0, 0.2, -1.3)]
    for i, (m, p) in enumerate(zip(mats, pos)):
        v, f = cube_mesh(p, 0.45, rot_y=0.3 * i)
        s.add_mesh(v, f, m)
    return s


def default_camera(res):
    """Camera::builder().build() at resolution `res` (camera/builder.rs defaults)."""
    return L.Camera.builder().resolution(res).build()
