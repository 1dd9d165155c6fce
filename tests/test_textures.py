"""Host side of textures (texture.rs, image.rs, perlin.rs, parser/mtl/task.rs): the decoded
texel tables the device samples, checked against Python restatements of lumo's decoders.

* Image::decode_png (image.rs:19-78) over every colour type / bit depth lumo reads, every PNG
  row filter, including lumo's index arithmetic for packed palettes (bytes read LSB-first with
  no row padding skipped) -- the PNGs are written here by a small zlib encoder;
* Image::from_file (image.rs:254-276): texels Spectrum::from_srgb, mean Spectrum::from_rgb of
  the mean linear RGB;
* Image::from_hdri_bytes (image.rs:205-252) with RGB::from_rgbe (rgb.rs:79-92, incl. its
  `0.5 +` offset);
* Image::bump_from_file (image.rs:142-169): normalize(c / 128 - 1);
* Perlin::new(seed) (perlin.rs:31-47, rng.rs:37-116, maps.rs:49-55);
* MTL map_Kd / map_Ke / map_Ks (both map_ks modes) / map_Bump (parser/mtl/task.rs, mtl.rs:60-90)
  with _extract_zip's case-insensitive suffix lookup (parser.rs:88-114).
No GPU needed; the device sampling is covered in test_gpu_textures.py.
"""
import io
import math
import zipfile

import numpy as np
import pytest

import lumo_amd as L
from imgdata import from_rgbe, hdr_bytes, png_bytes, random_png
from lumo_amd import _ffi


# ------------------------------------------------------------------ scene helpers
def _textured_scene(material, env=None):
    s = L.Scene()
    s.add_rectangle([0, 1, 0], [1, 1, 0], [1, 1, 1], L.Material.light(L.Spectrum.from_rgb(1, 1, 1)), light=True)
    s.add_rectangle([0, 0, 0], [1, 0, 0], [1, 0, 1], material)
    if env is not None:
        s.set_environment_map(env, 1.0)
    return s


def _tables(desc):
    tex = np.ctypeslib.as_array(desc.textures, shape=(desc.num_textures,)) if desc.num_textures else None
    texels = (np.ctypeslib.as_array(desc.texels, shape=(desc.num_texels,)) if desc.num_texels else None)
    return tex, texels


def _spec_tuple(s):
    s = s._s if isinstance(s, L.Spectrum) else s
    return (s["c0"], s["c1"], s["c2"], s["scale"]) if isinstance(s, np.void) else (s.c0, s.c1, s.c2, s.scale)


def srgb_decode(v):  # rgb.rs:59-66
    u = v / 255.0
    return u / 12.92 if u <= 0.04045 else ((u + 0.055) / 1.055) ** 2.4


def _texture_of(desc):
    mats = np.ctypeslib.as_array(desc.materials, shape=(desc.num_materials,))
    used = [m for m in mats if m["albedo_tex"] >= 0]
    assert len(used) == 1
    return used[0]


# ------------------------------------------------------------------ PNG
PNG_KINDS = [(2, 8), (6, 8), (0, 8), (4, 8), (3, 8), (3, 4), (3, 2), (3, 1)]


@pytest.mark.parametrize("ctype,bd", PNG_KINDS)
def test_png_texels_and_mean(ctype, bd):
    rng = np.random.default_rng(100 * ctype + bd)
    w, h = 7, 5  # odd width: packed rows carry padding bits
    data, px = random_png(rng, w, h, ctype, bd)
    sc = _textured_scene(L.Material.diffuse(L.Texture.image(data)))
    d = sc.desc()
    tex, texels = _tables(d)
    m = _texture_of(d)
    t = tex[m["albedo_tex"]]
    assert (t["kind"], t["width"], t["height"]) == (_ffi.TEX_IMAGE, w, h)
    got = texels[t["first"]:t["first"] + w * h]
    for g, p in zip(got, px):
        assert _spec_tuple(g) == _spec_tuple(L.Spectrum.from_srgb(*p))
    acc = [0.0, 0.0, 0.0]
    for p in px:  # image.rs:258-260: fold of RGB::from_srgb, then / len
        acc = [acc[k] + srgb_decode(p[k]) for k in range(3)]
    mean = L.Spectrum.from_rgb(*[a / len(px) for a in acc])
    assert _spec_tuple(t["spec"]) == _spec_tuple(mean)


@pytest.mark.parametrize("what", ["interlaced", "sixteen", "grey4", "corrupt"])
def test_png_rejections(what):
    rng = np.random.default_rng(5)
    if what == "interlaced":
        data = png_bytes(4, 4, 2, 8, [bytes(12)] * 4, interlace=1)
    elif what == "sixteen":
        data = png_bytes(4, 4, 2, 16, [bytes(24)] * 4)
    elif what == "grey4":
        data = png_bytes(4, 4, 0, 4, [bytes(2)] * 4)
    else:
        data, _ = random_png(rng, 4, 4, 2, 8)
        data = data[:40] + b"\x00" * 10 + data[50:]
    with pytest.raises(ValueError):
        _textured_scene(L.Material.diffuse(L.Texture.image(data))).build()


# ------------------------------------------------------------------ HDR
def test_hdr_environment_texels_and_mean():
    rng = np.random.default_rng(9)
    w, h = 6, 4
    px = rng.integers(0, 256, size=(w * h, 4))
    px[:, 3] = rng.integers(120, 136, size=w * h)
    px[3, 3] = 0  # e == 0: black
    sc = _textured_scene(L.Material.diffuse(L.Spectrum.from_rgb(0.5, 0.5, 0.5)),
                         env=L.Texture.hdr(hdr_bytes(w, h, px)))
    d = sc.desc()
    tex, texels = _tables(d)
    mats = np.ctypeslib.as_array(d.materials, shape=(d.num_materials,))
    env = [m for m in mats if m["albedo_tex"] >= 0]
    assert len(env) == 1 and env[0]["kind"] == _ffi.MAT_LIGHT
    t = tex[env[0]["albedo_tex"]]
    assert (t["kind"], t["width"], t["height"]) == (_ffi.TEX_IMAGE, w, h)
    acc = [0.0, 0.0, 0.0]
    for i, p in enumerate(px):
        rgb = from_rgbe(*[int(x) for x in p])
        assert _spec_tuple(texels[t["first"] + i]) == _spec_tuple(L.Spectrum.from_rgb(*rgb))
        acc = [acc[k] + rgb[k] for k in range(3)]
    mean = L.Spectrum.from_rgb(*[a / (w * h) for a in acc])
    assert _spec_tuple(t["spec"]) == _spec_tuple(mean)


@pytest.mark.parametrize("bad", [b"#?RGBE\n-Y 1 +X 1\n\x01\x01\x01\x80", b"#?RADIANCE\n-Y 2 +X 2\n\x01\x01\x01\x80",
                                 b"#?RADIANCE\n+X 1 -Y 1\n\x01\x01\x01\x80",
                                 # sizes whose product wraps to 0 (an empty body would pass the size
                                 # check) or overflows int32 texel indexing: rejected as lumo's u32 parse
                                 b"#?RADIANCE\n-Y 4 +X 4611686018427387904\n", b"#?RADIANCE\n-Y 65536 +X 65536\n"])
def test_hdr_rejections(bad):
    """image.rs:214-238 asserts: the magic line, the '-Y h +X w' order, w * h * 4 data bytes."""
    with pytest.raises(ValueError):
        _textured_scene(L.Material.diffuse(L.Spectrum.from_rgb(0.5, 0.5, 0.5)), env=L.Texture.hdr(bad)).build()


# ------------------------------------------------------------------ bump maps
def test_bump_map_normals():
    rng = np.random.default_rng(3)
    data, px = random_png(rng, 5, 3, 2, 8)
    sc = _textured_scene(L.Material.microfacet(0.5, 1.5, 0.0, False, False, L.Spectrum.from_rgb(0.5, 0.5, 0.5),
                                               L.Spectrum.from_rgb(1, 1, 1), L.Spectrum.black(),
                                               bump_map=L.NormalMap(data)))
    d = sc.desc()
    mats = np.ctypeslib.as_array(d.materials, shape=(d.num_materials,))
    used = [m for m in mats if m["normal_map"] >= 0]
    assert len(used) == 1
    nm = np.ctypeslib.as_array(d.normal_maps, shape=(d.num_normal_maps,))[used[0]["normal_map"]]
    assert (nm["width"], nm["height"]) == (5, 3)
    n = np.ctypeslib.as_array(d.normal_texels, shape=(d.num_normal_texels, 3))[nm["first"]:nm["first"] + 15]
    for got, p in zip(n, px):
        v = [c / 128.0 - 1.0 for c in p]
        ln = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])  # Vec3::normalize: self / length
        assert list(got) == [x / ln for x in v]


# ------------------------------------------------------------------ Perlin
def _xorshift(seed):
    M = (1 << 64) - 1
    st = [max(seed, 1), max(seed, 1)]  # lo, hi

    def step():
        lo, hi = st
        st[1] = lo
        hi ^= (hi << 23) & M
        hi ^= hi >> 17
        hi ^= lo
        st[0] = (hi + lo) & M
        return hi

    for _ in range(3):
        step()
    return step


def perlin_ref(seed):
    step = _xorshift(seed)

    def fl():
        return min(float(step()) * 2.0 ** -64, 1.0 - 1e-10)

    lattice = []
    for _ in range(256):
        x, y = fl(), fl()
        z = 1.0 - 2.0 * y
        r = math.sqrt(max(1.0 - z * z, 0.0))
        phi = 2.0 * math.pi * x
        lattice.append((r * math.cos(phi), r * math.sin(phi), z))
    perms = []
    for _ in range(3):
        p = list(range(256))
        for i in range(255):
            j = i + step() % (256 - i)
            p[i], p[j] = p[j], p[i]
        perms.append(p)
    return np.array(lattice), np.array(perms)


def test_perlin_lattice_and_permutations():
    sc = _textured_scene(L.Material.diffuse(L.Texture.marble(1234567, L.Spectrum.from_rgb(0.8, 0.7, 0.6))))
    d = sc.desc()
    assert d.num_perlin == 1
    p = d.perlin[0]
    lat = np.array([[p.lattice[i][k] for k in range(3)] for i in range(256)])
    perm = np.array([[p.perm[a][i] for i in range(256)] for a in range(3)])
    rl, rp = perlin_ref(1234567)
    np.testing.assert_array_equal(perm, rp)
    # cos / sin: the product's restated libm vs the platform's (<= 1 ulp apart)
    np.testing.assert_allclose(lat, rl, rtol=0, atol=4e-16)


def test_checkerboard_children_precede_parent():
    a, b = L.Texture.solid(L.Spectrum.from_rgb(1, 0, 0)), L.Texture.mandelbrot()
    cb = L.Texture.checkerboard(L.Texture.checkerboard(a, b, 3.0), a, 10.0)
    d = _textured_scene(L.Material.diffuse(cb)).desc()
    tex, _ = _tables(d)
    root = _texture_of(d)["albedo_tex"]
    assert tex[root]["kind"] == _ffi.TEX_CHECKERBOARD and tex[root]["scale"] == 10.0
    inner = tex[tex[root]["first"]]
    assert inner["kind"] == _ffi.TEX_CHECKERBOARD and inner["scale"] == 3.0
    assert tex[root]["second"] == inner["first"]  # the shared texture is registered once
    for i, t in enumerate(tex):
        if t["kind"] == _ffi.TEX_CHECKERBOARD:
            assert t["first"] < i and t["second"] < i


def test_textured_light_power_uses_image_mean():
    """Material::power -> Texture::power (texture.rs:95-101): image mean; marble is unimplemented!()."""
    data, _ = random_png(np.random.default_rng(1), 3, 3, 2, 8)
    s = L.Scene()
    s.add_rectangle([0, 1, 0], [1, 1, 0], [1, 1, 1], L.Material.light(L.Texture.image(data)), light=True)
    s.add_rectangle([0, 0, 0], [1, 0, 0], [1, 0, 1], L.Material.lambertian(L.Spectrum.from_rgb(0.5, 0.5, 0.5)))
    s.build()
    s2 = L.Scene()
    s2.add_rectangle([0, 1, 0], [1, 1, 0], [1, 1, 1],
                     L.Material.light(L.Texture.marble(1, L.Spectrum.from_rgb(1, 1, 1))), light=True)
    with pytest.raises(ValueError):
        s2.build()


# ------------------------------------------------------------------ MTL maps
OBJ = b"""mtllib scene.mtl
v 0 0 0
v 1 0 0
v 1 0 1
v 0 0 1
v 0 2 0
v 1 2 0
v 1 2 1
vt 0 0
vt 1 0
vt 1 1
vt 0 1
usemtl floor
f 1/1 2/2 3/3 4/4
usemtl lamp
f 5/1 6/2 7/3
"""


def _zip(files):
    bio = io.BytesIO()
    with zipfile.ZipFile(bio, "w") as z:
        for n, b in files.items():
            z.writestr(n, b)
    return bio.getvalue()


@pytest.mark.parametrize("map_ks", [False, True])
def test_mtl_texture_maps(tmp_path, map_ks):
    rng = np.random.default_rng(11)
    kd, _ = random_png(rng, 4, 4, 2, 8)
    ke, _ = random_png(rng, 2, 2, 6, 8)
    orm, orm_px = random_png(rng, 3, 3, 2, 8)
    bump, _ = random_png(rng, 4, 2, 2, 8)
    # Ns first: the statements apply in order, so map_Ks's ORM roughness replaces Ns's
    mtl = (b"newmtl floor\nNs 100\nKd 1 1 1\nmap_Kd Textures\\Floor_KD.png\nmap_Ks textures/orm.png\n"
           b"map_Bump textures/bump.png\n\nnewmtl lamp\nKe 0 0 0\nmap_Ke textures/lamp.png\n")
    z = tmp_path / "s.zip"
    z.write_bytes(_zip({"scene.obj": OBJ, "scene.mtl": mtl, "Scenes/Textures/floor_kd.png": kd,
                        "Scenes/textures/orm.png": orm, "Scenes/textures/bump.png": bump,
                        "Scenes/textures/lamp.png": ke}))
    sc = L.Scene.from_file(str(z), "scene.obj", map_ks=map_ks)
    d = sc.desc()
    mats = np.ctypeslib.as_array(d.materials, shape=(d.num_materials,))
    tex, _ = _tables(d)
    floor = [m for m in mats if m["normal_map"] >= 0]
    assert len(floor) == 1
    f = floor[0]
    assert tex[f["albedo_tex"]]["width"] == 4 and tex[f["albedo_tex"]]["kind"] == _ffi.TEX_IMAGE
    if map_ks:
        assert tex[f["ks_tex"]]["width"] == 3
    else:  # ORM mean: roughness = mean g / 256, k = mean b / 256 (image.rs:81-95)
        assert f["ks_tex"] == -1
        sc_ = 1.0 / 9.0
        acc = [0.0, 0.0, 0.0]
        for p in orm_px:
            acc = [acc[k] + sc_ * p[k] / 256.0 for k in range(3)]
        assert f["roughness"] == acc[1]
        assert _spec_tuple(f["ks"]) == _spec_tuple(L.Spectrum.from_rgb(1, 1, 1))
    lamp = [m for m in mats if m["kind"] == _ffi.MAT_LIGHT and m["albedo_tex"] >= 0]
    assert len(lamp) == 1 and tex[lamp[0]["albedo_tex"]]["width"] == 2
    assert d.num_lights == 1


def test_mtl_ambiguous_texture_name(tmp_path):
    kd, _ = random_png(np.random.default_rng(2), 2, 2, 2, 8)
    mtl = b"newmtl floor\nKd 1 1 1\nmap_Kd kd.png\nnewmtl lamp\nKe 1 1 1\n"
    z = tmp_path / "s.zip"
    z.write_bytes(_zip({"scene.obj": OBJ, "scene.mtl": mtl, "a/kd.png": kd, "b/kd.png": kd}))
    with pytest.raises(ValueError):
        L.Scene.from_file(str(z), "scene.obj")


# ------------------------------------------------------------------ oracle over the texture zoo
def test_oracle_renders_texture_zoo():
    """The oracle samples every texture kind without faults and the image is lit (the GPU
    comparison is test_gpu_textures.py)."""
    import oracle_ffi as O
    from scenes import default_camera, texture_zoo
    sc = texture_zoo().build()
    cam = default_camera((24, 16))
    tasks = L.make_tasks(24, 16, 4, 99)
    bufs, _, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 4)
    img = np.concatenate([b.reshape(-1, 4) for b in bufs])
    assert np.isfinite(img).all() and img[:, :3].sum() > 0.0
    bufs, _, _ = O.render_tasks(sc.desc(), cam.desc, tasks[:2], O.WAVEFRONT, 4, integrator=1, splats_out=[])
    assert all(np.isfinite(b).all() for b in bufs)


def test_checkerboard_of_one_colour_is_solid():
    """Checkerboard(A, A) samples A everywhere: renders bit-identical to the solid material."""
    import oracle_ffi as O
    from scenes import default_camera
    a = L.Spectrum.from_rgb(0.3, 0.6, 0.2)

    def scene(t):
        return L.Scene.empty_box(L.Spectrum.from_srgb(242, 242, 242), L.Material.diffuse(t),
                                 L.Material.diffuse(L.Spectrum.from_rgb(0.5, 0.5, 0.5))).build()
    cam = default_camera((16, 16))
    tasks = L.make_tasks(16, 16, 4, 5)
    b1, _, _ = O.render_tasks(scene(a).desc(), cam.desc, tasks, O.WAVEFRONT, 4)
    b2, _, _ = O.render_tasks(scene(L.Texture.checkerboard(a, a, 5.0)).desc(), cam.desc, tasks, O.WAVEFRONT, 4)
    for x, y in zip(b1, b2):
        np.testing.assert_array_equal(x, y)


def test_oracle_renders_textured_obj_zip(tmp_path):
    import oracle_ffi as O
    from scenes import default_camera, textured_obj_zip
    sc = L.Scene.from_file(str(textured_obj_zip(tmp_path / "s.zip")), "scene.obj").build()
    d = sc.desc()
    mats = np.ctypeslib.as_array(d.materials, shape=(d.num_materials,))
    assert (mats["normal_map"] >= 0).sum() == 1 and d.num_textures == 2 and d.num_lights == 2
    cam = default_camera((16, 16))
    bufs, _, _ = O.render_tasks(d, cam.desc, L.make_tasks(16, 16, 4, 3), O.WAVEFRONT, 4)
    assert sum(float(b.reshape(-1, 4)[:, :3].sum()) for b in bufs) > 0.0


def test_decoded_texels_match_the_file_decoders():
    """lumo_builder_texture_texels / normal_map_texels (a binding that holds lumo's decoded
    Image<Spectrum> / Image<Normal>) give the same tables, and the same oracle render, as the
    PNG decoders."""
    import oracle_ffi as O
    from scenes import default_camera
    rng = np.random.default_rng(21)
    kd_png, _ = random_png(rng, 6, 4, 2, 8)
    bump_png, _ = random_png(rng, 5, 3, 2, 8)

    def scene(kd, bump):
        return L.Scene.empty_box(L.Spectrum.from_srgb(242, 242, 242),
                                 L.Material.microfacet(0.5, 1.5, 0.0, False, False, kd, L.Spectrum.from_rgb(1, 1, 1),
                                                       L.Spectrum.black(), bump_map=bump),
                                 L.Material.diffuse(L.Spectrum.from_rgb(0.5, 0.5, 0.5))).build()
    a = scene(L.Texture.image(kd_png), L.NormalMap(bump_png))
    da = a.desc()
    tex, texels = _tables(da)
    t = [x for x in tex if x["kind"] == _ffi.TEX_IMAGE][0]
    arr = np.array([list(_spec_tuple(x)) for x in texels[t["first"]:t["first"] + 24]], dtype=np.float32)
    mean = L.Spectrum(_ffi.Spectrum(*_spec_tuple(t["spec"])))
    nm = np.ctypeslib.as_array(da.normal_maps, shape=(da.num_normal_maps,))[0]
    normals = np.ctypeslib.as_array(da.normal_texels, shape=(da.num_normal_texels, 3))[nm["first"]:nm["first"] + 15]
    b = scene(L.Texture.texels(6, 4, arr, mean), L.NormalMap.from_normals(5, 3, normals.copy()))
    db = b.desc()
    tb, texb = _tables(db)
    tt = [x for x in tb if x["kind"] == _ffi.TEX_IMAGE][0]
    assert _spec_tuple(tt["spec"]) == _spec_tuple(t["spec"])
    assert [_spec_tuple(x) for x in texb[tt["first"]:tt["first"] + 24]] == \
           [_spec_tuple(x) for x in texels[t["first"]:t["first"] + 24]]
    cam = default_camera((16, 16))
    tasks = L.make_tasks(16, 16, 4, 8)
    ra, _, _ = O.render_tasks(da, cam.desc, tasks, O.WAVEFRONT, 4)
    rb, _, _ = O.render_tasks(db, cam.desc, tasks, O.WAVEFRONT, 4)
    for x, y in zip(ra, rb):
        np.testing.assert_array_equal(x, y)
