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


def cube_obj(center, size, rot_y=0.0, uv_scale=2.0):
    """The cube of cube_mesh as .obj text with per-face texture coordinates (0..uv_scale, so the
    uvs wrap, hit.rs:61-68)."""
    v, faces = cube_mesh(center, size, rot_y)
    lines = [f"v {float(x)!r} {float(y)!r} {float(z)!r}" for x, y, z in v]
    s = uv_scale
    lines += [f"vt 0 0", f"vt {s!r} 0", f"vt {s!r} {s!r}", f"vt 0 {s!r}"]
    lines += ["f " + " ".join(f"{i + 1}/{k + 1}" for k, i in enumerate(f)) for f in faces]
    return ("\n".join(lines) + "\n").encode()


def texture_zoo(seed=7):
    """empty_box with every texture kind (texture.rs): checkerboard of marble / Mandelbrot and an
    image on the walls, image kd + bump map, image ks (metal), checkerboard tf (dielectric), a
    marble sphere, an image-textured light and a Radiance HDR environment map."""
    from imgdata import hdr_bytes, random_png
    rng = np.random.default_rng(seed)
    img = L.Texture.image(random_png(rng, 13, 9, 2, 8)[0])
    pal = L.Texture.image(random_png(rng, 8, 8, 3, 4)[0])
    bump = L.NormalMap(random_png(rng, 6, 5, 2, 8)[0])
    marble = L.Texture.marble(1234, L.Spectrum.from_rgb(0.8, 0.75, 0.7))
    checker = L.Texture.checkerboard(marble, L.Texture.mandelbrot(), 6.0)
    s = L.Scene.empty_box(L.Spectrum.from_srgb(242, 242, 242), L.Material.diffuse(checker), L.Material.diffuse(img))
    objs = [(L.Material.microfacet(0.4, 1.5, 0.0, False, False, pal, L.Spectrum.from_rgb(1, 1, 1),
                                   L.Spectrum.black(), bump_map=bump), (-0.55, -0.55, -1.5)),
            (L.Material.metal(img, 0.25, 1.5, 3.0), (0.55, -0.55, -1.5)),
            (L.Material.transparent(L.Texture.checkerboard(L.Spectrum.from_rgb(0.9, 0.6, 0.6),
                                                           L.Spectrum.from_rgb(0.6, 0.9, 0.9), 3.0), 0.2, 1.5),
             (0.0, -0.55, -1.0))]
    for i, (m, p) in enumerate(objs):
        s.add_obj(cube_obj(p, 0.45, rot_y=0.4 * i), m)
    s.add_sphere(0.2, L.Material.diffuse(marble)).translate(0.0, 0.25, -1.6)
    s.add_rectangle([-0.25, 0.79, -1.4], [0.25, 0.79, -1.4], [0.25, 0.79, -0.9],
                    L.Material.light(L.Texture.image(random_png(rng, 4, 4, 6, 8)[0]), scale=4.0), light=True)
    px = rng.integers(0, 256, size=(8 * 4, 4))
    px[:, 3] = rng.integers(126, 131, size=32)
    s.set_environment_map(L.Texture.hdr(hdr_bytes(8, 4, px)), 0.5)
    return s


def textured_obj_zip(path):
    """A zip with an .obj (textured cube, floor, emissive quad), its .mtl using map_Kd (named
    with a backslash and other case), map_Bump and map_Ke, and the PNGs; returns `path`."""
    import io
    import zipfile

    from imgdata import random_png
    rng = np.random.default_rng(4)
    files = {"t/kd.png": random_png(rng, 9, 7, 2, 8)[0], "t/bump.png": random_png(rng, 5, 5, 2, 8)[0],
             "t/lamp.png": random_png(rng, 3, 3, 6, 8)[0]}
    obj = cube_obj((0.0, -0.3, -1.5), 0.6, 0.5).decode().replace("f ", "usemtl box\nf ", 1)
    nv = 8
    obj += ("v -0.3 0.7 -1.8\nv 0.3 0.7 -1.8\nv 0.3 0.7 -1.2\nv -0.3 0.7 -1.2\n"
            f"usemtl lamp\nf {nv + 1}/1 {nv + 2}/2 {nv + 3}/3 {nv + 4}/4\n")
    obj += ("v -5 -0.6 -5\nv 5 -0.6 -5\nv 5 -0.6 5\nv -5 -0.6 5\n"
            f"usemtl box\nf {nv + 8}/1 {nv + 7}/2 {nv + 6}/3 {nv + 5}/4\n")
    mtl = (b"newmtl box\nKd 0.8 0.8 0.8\nNs 200\nmap_Kd T\\KD.png\nmap_Bump t/bump.png\n"
           b"newmtl lamp\nKe 1 1 1\nmap_Ke t/lamp.png\n")
    bio = io.BytesIO()
    with zipfile.ZipFile(bio, "w") as z:
        z.writestr("scene.obj", "mtllib scene.mtl\n" + obj)
        z.writestr("scene.mtl", mtl)
        for n, b in files.items():
            z.writestr(n, b)
    path.write_bytes(bio.getvalue())
    return path
