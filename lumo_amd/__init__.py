"""lumo_amd — MI355X (gfx950) wavefront path tracer with lumo's API.

Python mirror of lumo's builder API (ekarpp/lumo v0.6.1) over the C ABI in include/:
    Spectrum.from_rgb / from_srgb / from_pts          (src/tracer/color/spectrum.rs)
    Material.lambertian / Material.light               (src/tracer/material.rs)
    Scene() .add_mesh / .add_rectangle / cornell_box() (src/tracer/scene.rs, scene/cornell_box.rs)
    Camera.builder() ... .build(), Camera.cornell_box()(src/tracer/camera*.rs)
    Renderer(scene, camera).samples(n).seed(s).render() -> Film   (src/renderer.rs)

Scene construction runs in the C++ host library; rendering runs only on the GPU through
lumo_render_tiles (the replacement of lumo's RenderTaskExecutor::exec).  There is no CPU
fallback: without a gfx950 device, Renderer.render raises.
"""
import ctypes as C

import numpy as np

from . import _ffi
from ._ffi import check

__all__ = ["Spectrum", "Texture", "NormalMap", "Material", "Scene", "Camera", "Renderer", "Integrator", "ToneMap", "Film", "Device",
           "DENSE", "TILE_SIZE", "SAMPLES_INCREMENT", "make_tasks"]

TILE_SIZE = 16          # renderer.rs:15
SAMPLES_INCREMENT = 256  # renderer.rs:17
DENSE = {"CIE_X": 0, "CIE_Y": 1, "CIE_Z": 2, "A": 3, "D50": 4, "D65": 5, "F2": 6, "F7": 7, "CORNELL": 8,
         "GLASS_ETA": 9, "DIAMOND_ETA": 10, "MIRROR_ETA": 11, "MIRROR_K": 12}


def lib():
    return _ffi.load()


class Spectrum:
    """Sigmoid-polynomial spectrum (spectrum.rs:14-19): c0, c1, c2 (f32) and scale."""

    def __init__(self, s):
        self._s = s

    @staticmethod
    def from_rgb(r, g, b):
        return Spectrum(lib().lumo_spectrum_from_rgb(r, g, b))

    @staticmethod
    def from_srgb(r, g, b):
        return Spectrum(lib().lumo_spectrum_from_srgb(r, g, b))

    @staticmethod
    def from_pts(pts):
        return Spectrum(lib().lumo_spectrum_from_pts(pts.encode()))

    @property
    def coeffs(self):
        return (self._s.c0, self._s.c1, self._s.c2)

    @property
    def scale(self):
        return self._s.scale

    def is_black(self):
        return self._s.scale == 0.0


    @staticmethod
    def black():
        return Spectrum(_ffi.Spectrum(0.0, 0.0, 0.0, 0.0))


# spectrum.rs:22-38 constants, built on first use (they need the library's rgb2spec table)
_NAMED = {"WHITE": (1.0, 1.0, 1.0), "RED": (1.0, 0.0, 0.0), "GREEN": (0.0, 1.0, 0.0), "BLUE": (0.0, 0.0, 1.0),
          "YELLOW": (1.0, 1.0, 0.0), "MAGENTA": (1.0, 0.0, 1.0), "CYAN": (0.0, 1.0, 1.0)}


def named_spectrum(name):
    """Spectrum::WHITE / BLACK / RED / GREEN / BLUE / YELLOW / MAGENTA / CYAN."""
    if name == "BLACK":
        return Spectrum.black()
    return Spectrum.from_rgb(*_NAMED[name])


class Texture:
    """lumo's Texture (texture.rs:23-92): Solid / Checkerboard / Marble / Image / Mandelbrot.
    Registered with a scene's builder when a material (or the environment map) using it is
    added; anywhere a Texture is accepted a Spectrum means Texture::Solid."""

    def __init__(self, kind, **kw):
        self.kind, self.kw = kind, kw

    @staticmethod
    def solid(spec):
        return Texture("solid", spec=spec)

    @staticmethod
    def image(source):
        """Texture::Image(Image::from_path / from_file): a PNG as a path, bytes, or (zip, member)."""
        return Texture("image", data=_read_source(source, ".png"))

    @staticmethod
    def hdr(source):
        """Texture::Image(Image::from_hdri_bytes): a Radiance .hdr (flat RGBE) image."""
        return Texture("hdr", data=_read_source(source, ".hdr"))

    @staticmethod
    def texels(width, height, spectra, mean):
        """An already decoded Image<Spectrum>: width x height Spectra (row-major from the top row,
        as Image::buffer) or an (N, 4) float32 array of (c0, c1, c2, scale), and the mean Spectrum."""
        arr = np.ascontiguousarray(
            [(x._s.c0, x._s.c1, x._s.c2, x._s.scale) for x in spectra] if not isinstance(spectra, np.ndarray)
            else spectra, dtype=np.float32).reshape(-1, 4)
        if len(arr) != width * height:
            raise ValueError("texels: width * height spectra expected")
        return Texture("texels", width=int(width), height=int(height), arr=arr, mean=mean)

    @staticmethod
    def checkerboard(even, odd, scale):
        """Texture::Checkerboard(even, odd, scale): `even` where floor(u s) + floor(v s) is even."""
        return Texture("checkerboard", even=_as_texture(even), odd=_as_texture(odd), scale=float(scale))

    @staticmethod
    def marble(seed, spec):
        """Texture::Marble(Perlin::new(seed), spec)."""
        return Texture("marble", seed=int(seed), spec=spec)

    @staticmethod
    def mandelbrot():
        return Texture("mandelbrot")

    def _solid_spec(self):
        return self.kw["spec"] if self.kind == "solid" else None

    def _add(self, b, cache):
        """Index of this texture in builder b; `cache` (owned by the Scene) registers it once."""
        if id(self) in cache:
            return cache[id(self)][1]
        L, k = lib(), self.kw
        if self.kind == "solid":
            i = L.lumo_builder_texture_solid(b, k["spec"]._s)
        elif self.kind == "image":
            i = L.lumo_builder_texture_image(b, k["data"], len(k["data"]))
        elif self.kind == "hdr":
            i = L.lumo_builder_texture_hdr(b, k["data"], len(k["data"]))
        elif self.kind == "texels":
            i = L.lumo_builder_texture_texels(b, k["width"], k["height"],
                                              k["arr"].ctypes.data_as(C.POINTER(_ffi.Spectrum)), k["mean"]._s)
        elif self.kind == "checkerboard":
            i = L.lumo_builder_texture_checkerboard(b, k["even"]._add(b, cache), k["odd"]._add(b, cache), k["scale"])
        elif self.kind == "marble":
            i = L.lumo_builder_texture_marble(b, k["seed"], k["spec"]._s)
        else:
            i = L.lumo_builder_texture_mandelbrot(b)
        if i < 0:
            raise ValueError(f"texture {self.kind}: " + L.lumo_builder_error(b).decode())
        cache[id(self)] = (self, i)
        return i


class NormalMap:
    """A bump map, Image<Normal> (image.rs:142-166): n = normalize(rgb / 128 - 1) of a PNG."""

    def __init__(self, source):
        self.data = _read_source(source, ".png") if source is not None else None
        self.normals = None

    @staticmethod
    def from_normals(width, height, normals):
        """An already decoded Image<Normal>: width x height unit normals (N, 3), row-major."""
        nm = NormalMap(None)
        nm.normals = np.ascontiguousarray(normals, dtype=np.float64).reshape(-1, 3)
        if len(nm.normals) != width * height:
            raise ValueError("normal map: width * height normals expected")
        nm.size = (int(width), int(height))
        return nm

    def _add(self, b, cache):
        if id(self) not in cache:
            if self.normals is not None:
                i = lib().lumo_builder_normal_map_texels(b, self.size[0], self.size[1],
                                                         self.normals.ctypes.data_as(_ffi.c_double_p))
            else:
                i = lib().lumo_builder_normal_map(b, self.data, len(self.data))
            if i < 0:
                raise ValueError("normal map: " + lib().lumo_builder_error(b).decode())
            cache[id(self)] = (self, i)
        return cache[id(self)][1]


def _as_texture(t):
    return t if isinstance(t, Texture) else Texture.solid(t)


def _split(t):
    """(solid spectrum for the material slot, texture or None)"""
    t = _as_texture(t)
    spec = t._solid_spec()
    return (spec, None) if spec is not None else (Spectrum.black(), t)


class Material:
    def __init__(self, kind, **kw):
        self.kind = kind
        self.kw = kw

    @staticmethod
    def lambertian(spec):
        return Material("lambertian", spec=spec)

    @staticmethod
    def light(tex, illuminant="D65", scale=1.0, two_sided=False):
        """Material::Light(texture, illuminant, scale, two_sided); Material::light uses D65.
        `tex` a Spectrum (solid) or an image Texture (power = the image mean, image.rs:187-189)."""
        return Material("light", spec=tex, illuminant=illuminant, scale=scale, two_sided=two_sided)

    @staticmethod
    def microfacet(roughness, eta, k, is_transparent, fresnel_enabled, kd, ks, tf, bump_map=None):
        """Material::microfacet (material.rs:26-68): kd / ks / tf Textures (or Spectra), an
        optional NormalMap bump map."""
        return Material("microfacet", roughness=roughness, eta=eta, k=k, is_transparent=is_transparent,
                        fresnel_enabled=fresnel_enabled, kd=kd, ks=ks, tf=tf, bump_map=bump_map)

    @staticmethod
    def diffuse(kd):
        """Material::diffuse: MfDiffuse, roughness 1 (material.rs:94-115)."""
        return Material("diffuse", kd=kd)

    @staticmethod
    def metal(ks, roughness, eta, k):
        """Material::metal: MfConductor (material.rs:71-91)."""
        return Material("metal", ks=ks, roughness=roughness, eta=eta, k=k)

    @staticmethod
    def transparent(tf, roughness, eta):
        """Material::transparent: MfDielectric (material.rs:123-143)."""
        return Material("transparent", tf=tf, roughness=roughness, eta=eta)

    @staticmethod
    def mirror():
        return Material("mirror")

    @staticmethod
    def glass():
        return Material("glass")

    def _add(self, b, cache=None):
        """Add to builder b: the material with the solid slots, then (when a slot holds a
        non-solid texture or there is a bump map) its textured copy."""
        k = dict(self.kw)
        tex = {}
        for slot in ("kd", "ks", "tf", "spec"):
            if slot in k and not (self.kind == "lambertian"):
                k[slot], t = _split(k[slot])
                if t is not None:
                    tex[slot] = t
        base = self._add_solid(b, k)
        nm = k.get("bump_map")
        if base < 0 or (not tex and nm is None):
            return base
        cache = {} if cache is None else cache
        ti = {s: t._add(b, cache) for s, t in tex.items()}
        albedo = ti.get("kd", ti.get("spec", -1))
        return lib().lumo_builder_material_textured(b, base, albedo, ti.get("ks", -1), ti.get("tf", -1),
                                                    nm._add(b, cache) if nm is not None else -1)

    def _add_solid(self, b, k):
        L = lib()
        if self.kind == "lambertian":
            return L.lumo_builder_material_lambertian(b, k["spec"]._s)
        if self.kind == "microfacet":
            return L.lumo_builder_material_microfacet(b, k["roughness"], k["eta"], k["k"], int(k["is_transparent"]),
                                                      int(k["fresnel_enabled"]), k["kd"]._s, k["ks"]._s, k["tf"]._s)
        if self.kind == "diffuse":
            return L.lumo_builder_material_diffuse(b, k["kd"]._s)
        if self.kind == "metal":
            return L.lumo_builder_material_metal(b, k["ks"]._s, k["roughness"], k["eta"], k["k"])
        if self.kind == "transparent":
            return L.lumo_builder_material_transparent(b, k["tf"]._s, k["roughness"], k["eta"])
        if self.kind == "mirror":
            return L.lumo_builder_material_mirror(b)
        if self.kind == "glass":
            return L.lumo_builder_material_glass(b)
        ill = k["illuminant"]
        ill = DENSE[ill] if isinstance(ill, str) else int(ill)
        return L.lumo_builder_material_light(b, k["spec"]._s, ill, float(k["scale"]), int(bool(k["two_sided"])))


def _read_source(source, suffix):
    """bytes of a file: raw bytes, a path, or (zip path, member name) -- the member is matched
    case-insensitively by suffix like parser.rs::_extract_zip."""
    if isinstance(source, (bytes, bytearray)):
        return bytes(source)
    if isinstance(source, tuple):
        import zipfile
        zpath, member = source
        with zipfile.ZipFile(zpath) as z:
            hits = [n for n in z.namelist() if n.lower().endswith((member or suffix).lower())]
            if len(hits) != 1:
                raise ValueError(f"{len(hits)} files matching {member or suffix} in {zpath}")
            return z.read(hits[0])
    with open(source, "rb") as f:
        return f.read()


class ObjectRef:
    """Handle to an object added to a Scene; Instanceable transformations compose in call order
    (object/instance.rs:203-299): mesh.to_unit_size().to_origin().rotate_y(a).translate(x, y, z)."""
    _OPS = {"translate": 0, "scale": 1, "rotate_x": 2, "rotate_y": 3, "rotate_z": 4, "to_unit_size": 5,
            "to_origin": 6, "set_x": 7, "set_y": 8, "set_z": 9}

    def __init__(self, scene, index, light=False):
        self.scene, self.index, self.light = scene, index, light

    def _op(self, name, x=0.0, y=0.0, z=0.0):
        check(lib().lumo_builder_instance_op(self.scene._b, int(self.light), self.index, self._OPS[name], x, y, z),
              name)
        self.scene._flat = None
        return self

    def translate(self, x, y, z):
        return self._op("translate", x, y, z)

    def scale(self, x, y, z):
        return self._op("scale", x, y, z)

    def scale_uniform(self, s):
        return self._op("scale", s, s, s)

    def rotate_x(self, r):
        return self._op("rotate_x", r)

    def rotate_y(self, r):
        return self._op("rotate_y", r)

    def rotate_z(self, r):
        return self._op("rotate_z", r)

    def to_unit_size(self):
        return self._op("to_unit_size")

    def to_origin(self):
        return self._op("to_origin")

    def set_x(self, v):
        return self._op("set_x", v)

    def set_y(self, v):
        return self._op("set_y", v)

    def set_z(self, v):
        return self._op("set_z", v)


class Scene:
    """lumo Scene: objects + lights; build() produces the flattened device image."""

    def __init__(self, _builder=None):
        L = lib()
        self._b = _builder if _builder is not None else L.lumo_builder_new()
        self._flat = None
        self._tex = {}  # id(Texture / NormalMap) -> (object, index in this builder)

    @staticmethod
    def cornell_box():
        return Scene(lib().lumo_builder_cornell_box())

    @staticmethod
    def empty_box(def_color, mat_left, mat_right):
        """Scene::empty_box (scene/empty_box.rs): 2 x 1.6 x 2 box centred at (0, 0, -1), one
        small ceiling light, MfDiffuse floor / roof / front wall of `def_color`."""
        s = Scene()
        ml, mr = s._mat(mat_left), s._mat(mat_right)
        check(lib().lumo_builder_empty_box(s._b, def_color._s, ml, mr), "empty_box")
        return s

    def _mat(self, m):
        idx = m._add(self._b, self._tex)
        if idx < 0:
            raise ValueError("invalid material")
        return idx

    def add_mesh(self, vertices, faces, material, light=False):
        """TriangleMesh::new(vertices, faces, [], [], material) added with Scene::add."""
        v = np.ascontiguousarray(np.asarray(vertices, dtype=np.float64).reshape(-1, 3))
        if isinstance(faces, np.ndarray) and faces.ndim == 2:  # uniform polygons, fast path
            idx = np.ascontiguousarray(faces, dtype=np.int64).reshape(-1)
            sizes = np.full(len(faces), faces.shape[1], dtype=np.int64)
        else:
            sizes = np.asarray([len(f) for f in faces], dtype=np.int64)
            idx = np.asarray([i for f in faces for i in f], dtype=np.int64)
        m = self._mat(material)
        st = lib().lumo_builder_add_mesh(self._b, v.ctypes.data_as(_ffi.c_double_p), len(v),
                                         idx.ctypes.data_as(_ffi.c_int64_p), sizes.ctypes.data_as(_ffi.c_int64_p),
                                         len(sizes), m, int(light))
        check(st, "add_mesh")
        self._flat = None
        if light:  # one Triangle light per face triangle (parser/obj.rs:93-103)
            return None
        return ObjectRef(self, lib().lumo_builder_count(self._b, 0) - 1)

    def add_rectangle(self, a, b, c, material, light=False):
        """Rectangle::new(Mat3::new(a, b, c), material) via Scene::add / Scene::add_light."""
        arr = [np.ascontiguousarray(np.asarray(x, dtype=np.float64)) for x in (a, b, c)]
        m = self._mat(material)
        st = lib().lumo_builder_add_rectangle(self._b, *[x.ctypes.data_as(_ffi.c_double_p) for x in arr], m,
                                              int(light))
        check(st, "add_rectangle")
        self._flat = None
        return ObjectRef(self, lib().lumo_builder_count(self._b, int(light)) - 1, light)

    def add_obj(self, source, material):
        """parser::mesh_from_path / mesh_from_url (parser.rs): the .obj (path, bytes, or
        (zip path, member suffix)) as one TriangleMesh with `material`; returns an ObjectRef."""
        data = _read_source(source, ".obj")
        m = self._mat(material)
        idx = lib().lumo_builder_add_obj_mesh(self._b, data, len(data), m)
        if idx < 0:
            raise ValueError("obj: " + lib().lumo_builder_error(self._b).decode())
        self._flat = None
        return ObjectRef(self, idx)

    @staticmethod
    def from_file(path, obj_name=None, mtllib=None, map_ks=False, env_map=None):
        """parser::scene_from_file (parser.rs:203-265): `path` a .zip holding `obj_name` (and
        `mtllib`), or a plain .obj path with an optional .mtl path (texture files then resolve
        relative to the .mtl's directory).  One mesh per usemtl group; emissive groups become
        Triangle lights; map_Kd / map_Ke / map_Ks / map_Bump read the archive's PNGs (map_ks as in
        MtlTaskExecutor); env_map = (member name, scale) sets a Radiance .hdr environment."""
        import os
        s = Scene()
        L = lib()
        if str(path).lower().endswith(".zip"):
            import zipfile
            obj = _read_source((path, obj_name), ".obj")
            mtl = _read_source((path, mtllib), ".mtl") if mtllib else None
            with zipfile.ZipFile(path) as z:
                for n in z.namelist():
                    if not n.endswith("/") and not n.lower().endswith((".obj", ".mtl")):
                        data = z.read(n)
                        check(L.lumo_builder_add_file(s._b, n.encode(), data, len(data)), "add_file")
            env = (_read_source((path, env_map[0]), ".hdr"), env_map[1]) if env_map else None
        else:
            obj = _read_source(path, ".obj")
            mtl = _read_source(mtllib, ".mtl") if mtllib else None
            base = os.path.dirname(os.path.abspath(mtllib if mtllib else path))
            env = (_read_source(env_map[0], ".hdr"), env_map[1]) if env_map else None
        # parser.rs:219-249: the explicit mtllib, then every `mtllib` statement of the .obj
        mtls = [mtl] if mtl else []
        for line in obj.decode("utf-8", "replace").splitlines():
            tok = line.split()
            if len(tok) >= 2 and tok[0] == "mtllib":
                name = tok[1]
                if str(path).lower().endswith(".zip"):
                    mtls.append(_read_source((path, name), ".mtl"))
                else:  # plain files (not a lumo mode): follow the statement when the file is there
                    f = os.path.join(os.path.dirname(os.path.abspath(path)), name)
                    if os.path.exists(f):
                        mtls.append(_read_source(f, ".mtl"))
        mtl = b"\n".join(mtls) if mtls else None
        if not str(path).lower().endswith(".zip") and mtl:
            # plain files: register only the files the MTL's map statements name (matched by
            # _extract_zip's case-insensitive suffix rule under the MTL's directory), so the
            # directory's other images are never read
            wanted = set()
            for line in mtl.decode("utf-8", "replace").splitlines():
                tok = line.split()
                if len(tok) >= 2 and (tok[0].lower().startswith("map_") or tok[0].lower() in ("bump", "norm")):
                    wanted.add(tok[-1].replace("\\", "/").lower())
            for root, _, files in os.walk(base) if wanted else ():
                for f in files:
                    full = os.path.join(root, f)
                    rel = os.path.relpath(full, base).replace(os.sep, "/")
                    if any(rel.lower().endswith(w) for w in wanted):
                        with open(full, "rb") as fh:
                            data = fh.read()
                        check(L.lumo_builder_add_file(s._b, rel.encode(), data, len(data)), "add_file")
        check(L.lumo_builder_set_map_ks(s._b, int(bool(map_ks))), "map_ks")
        st = L.lumo_builder_load_obj_scene(s._b, obj, len(obj), mtl, len(mtl) if mtl else 0)
        if st != _ffi.LUMO_OK:
            raise ValueError("obj scene: " + L.lumo_builder_error(s._b).decode())
        if env is not None:
            s.set_environment_map(Texture("hdr", data=env[0]), env[1])
        return s

    def add_sphere(self, radius, material, light=False):
        """Sphere::new(radius, material) at the origin (object/sphere.rs); returns an ObjectRef
        for translate / scale (Instanceable)."""
        m = self._mat(material)
        check(lib().lumo_builder_add_sphere(self._b, float(radius), m, int(light)), "add_sphere")
        self._flat = None
        return ObjectRef(self, lib().lumo_builder_count(self._b, int(light)) - 1, light)

    def set_environment_map(self, tex, scale):
        """Scene::set_environment_map (scene.rs:73-78): a Spectrum (constant) or an image / HDR
        Texture on the environment sphere."""
        spec, t = _split(tex)
        if t is None:
            check(lib().lumo_builder_set_environment_map(self._b, spec._s, float(scale)), "environment map")
        else:
            check(lib().lumo_builder_set_environment_texture(self._b, t._add(self._b, self._tex), float(scale)),
                  "environment map")
        self._flat = None

    def build(self):
        if self._flat is None:
            p = lib().lumo_builder_build(self._b)
            if not p:
                raise ValueError("scene build failed (no lights?)")
            self._flat = C.c_void_p(p)
        return self

    def desc(self):
        self.build()
        d = _ffi.SceneDesc()
        check(lib().lumo_scene_get_desc(self._flat, C.byref(d)), "scene desc")
        d._owner = self  # the descriptor points into this scene's flat arrays
        return d

    def __del__(self):
        try:
            L = _ffi._lib
            if L is not None:
                if self._flat is not None:
                    L.lumo_scene_free(self._flat)
                L.lumo_builder_free(self._b)
        except Exception:
            pass


class Camera:
    class Builder:
        def __init__(self, params):
            self.p = params

        def origin(self, x, y, z):
            self.p.origin[:] = [x, y, z]
            return self

        def towards(self, x, y, z):
            self.p.towards[:] = [x, y, z]
            return self

        def up(self, x, y, z):
            self.p.up[:] = [x, y, z]
            return self

        def zoom(self, z):
            self.p.zoom = z
            return self

        def lens_radius(self, r):
            self.p.lens_radius = r
            return self

        def focal_length(self, f):
            self.p.focal_length = f
            return self

        def resolution(self, wh):
            self.p.width, self.p.height = int(wh[0]), int(wh[1])
            return self

        def vfov(self, v):
            self.p.vfov = v
            return self

        def illuminant(self, name):
            self.p.illuminant = DENSE[name] if isinstance(name, str) else int(name)
            return self

        def camera_type(self, t):
            """CameraType (camera/builder.rs:4-9): CameraType.Perspective or CameraType.Orthographic."""
            self.p.camera_type = int(t)
            return self

        def color_space(self, cs):
            """0 sRGB, 1 DCI-P3 (default), 2 Rec. 2020 (color/space.rs)."""
            self.p.color_space = int(cs)
            return self

        def build(self):
            d = _ffi.CameraDesc()
            check(lib().lumo_camera_build(C.byref(self.p), C.byref(d)), "camera build")
            cam = Camera(d, (self.p.width, self.p.height))
            cam.color_space = self.p.color_space
            return cam

    def __init__(self, desc, resolution, color_space=1):
        self.desc = desc
        self.resolution = resolution
        self.color_space = color_space

    @staticmethod
    def builder():
        p = _ffi.CameraParams()
        lib().lumo_camera_params_default(C.byref(p))
        return Camera.Builder(p)

    @staticmethod
    def cornell_box_builder():
        p = _ffi.CameraParams()
        lib().lumo_camera_params_cornell_box(C.byref(p))
        return Camera.Builder(p)

    @staticmethod
    def cornell_box(resolution=(512, 512)):
        return Camera.cornell_box_builder().resolution(resolution).build()


class CameraType:
    """camera/builder.rs:4-9."""
    Perspective = 0
    Orthographic = 1


class SamplerType:
    """samplers.rs:6-17: the pixel sampler of Renderer::sampler (renderer.rs:89-93)."""
    MultiJittered = 0  # lumo's default
    Uniform = 1
    Jittered = 2
    Sobol = 3  # at most 1023 samples per pixel (sobol_seq.rs SOBOL_MAX_LEN)


class Integrator:
    """integrator.rs:14-28: PathTrace (NEE + MIS) or BDPathTrace (bidirectional, MIS)."""
    PathTrace = 0
    BDPathTrace = 1


class ToneMap:
    """tone_mapping.rs: (kind, arg) pairs applied per sample before the film."""
    NO_MAP = (0, 0.0)
    REINHARD = (2, 0.0)

    @staticmethod
    def clamp(mx):
        return (1, float(mx))


def make_tasks(width, height, samples, seed):
    """renderer.rs:179-204: (batch, tile) tasks in publish order with their stream seeds."""
    L = lib()
    n = L.lumo_make_tasks(width, height, samples, seed, None, 0)
    arr = (_ffi.TileTask * n)()
    L.lumo_make_tasks(width, height, samples, seed, arr, n)
    return arr


class Film:
    """Film pixels (film.rs:57-92): per pixel sum of w*rgb and sum of w (PIXEL_BUFFERS = 1)."""

    def __init__(self, width, height, color_space=1, samples=1, filter_radius=1.5, filter_sigma=0.375):
        self.width, self.height = width, height
        self.color_space = color_space  # the camera's ColorSpace (default DCI-P3)
        self.pixels = np.zeros((height, width, 4), dtype=np.float64)
        self.splats = np.zeros((height, width, 3), dtype=np.float64)  # BDPT light tracing (film.rs:136)
        self.splat_scale = 1.0 / samples  # film.rs:137
        self.filter_radius, self.filter_sigma = filter_radius, filter_sigma

    def add_tile(self, task, rgb_w, splats=None):
        """Film::add_tile (film.rs:155-171): tile pixels, then the tile's splats in order."""
        x0, y0 = task.px_min[0], task.px_min[1]
        x1, y1 = task.px_max[0], task.px_max[1]
        self.pixels[y0:y1, x0:x1, :] += rgb_w.reshape(y1 - y0, x1 - x0, 4)
        if splats is not None:
            for sp in splats:  # sequential, in lumo's order
                self.splats[sp["y"], sp["x"]] += sp["rgb"]

    def filter_integral(self):
        """PixelFilter::integral for the Gaussian (filter.rs:103-114)."""
        import math
        r, s = self.filter_radius, self.filter_sigma
        denom = s * math.sqrt(2.0)
        ig = 0.5 * (math.erf(r / denom) - math.erf(-r / denom))
        gr = math.exp(-(r * r) / (2.0 * s * s)) / math.sqrt(max(2.0 * math.pi * s * s, 0.0))
        return (ig - 2.0 * r * gr) ** 2

    def rgb(self):
        """Pixel::value (film.rs:82-91) + splat_scale * splat / filter integral (film.rs:173-182)."""
        with np.errstate(invalid="ignore", divide="ignore"):
            direct = self.pixels[..., :3] / self.pixels[..., 3:4]
        if not self.splats.any():
            return direct
        return direct + self.splat_scale * self.splats / self.filter_integral()

    def rgb_image(self):
        """Film::rgb_image (film.rs:173-192): encoded 8-bit RGB, rows top to bottom."""
        from .image import encode
        return encode(self.rgb(), self.color_space)

    def save(self, path):
        """Film::save (film.rs:195-210): 8-bit RGB PNG."""
        from .image import write_png
        write_png(path, self.rgb_image())


class Device:
    """One lumo_amd context bound to one GPU (lumo_create)."""

    def __init__(self, device=0, **options):
        L = lib()
        ctx = C.c_void_p()
        st = L.lumo_create(device, C.byref(ctx))
        if st != _ffi.LUMO_OK:
            raise RuntimeError(f"lumo_create(device={device}) failed: {L.lumo_status_str(st).decode()}")
        self.ctx = ctx
        self.scene = None
        for k, v in options.items():  # execution options (LUMO_OPT_*), e.g. Device(0, split_pipe=1)
            self.set_option(k, v)

    def upload(self, scene, camera=None):
        L = lib()
        self._scene_desc = scene.desc()
        check(L.lumo_scene_upload(self.ctx, C.byref(self._scene_desc)), "scene upload")
        if camera is not None:
            check(L.lumo_camera_set(self.ctx, C.byref(camera.desc)), "camera set")
        self.scene = scene

    @staticmethod
    def _result_buffers(arr, n):
        """Per-task {Σw·rgb, Σw} buffers (4 f64 per tile pixel) as views of one allocation, with
        the lumo_tile_result array pointing at them.  Vectorised over the task array's fields
        (all u64): a per-task Python loop cost ~0.2 s per 16k-task frame, inside the timed step."""
        res = (_ffi.TileResult * n)()
        if n == 0:
            return [], [], res
        tv = np.frombuffer(arr, dtype=np.uint64).reshape(n, C.sizeof(_ffi.TileTask) // 8)
        if (tv[:, 2] < tv[:, 0]).any() or (tv[:, 3] < tv[:, 1]).any():
            raise ValueError("tile task with px_max < px_min")
        P = ((tv[:, 2] - tv[:, 0]) * (tv[:, 3] - tv[:, 1])).astype(np.int64)
        off = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(4 * P, out=off[1:])
        big = np.zeros(int(off[-1]), dtype=np.float64)
        rv = np.frombuffer(res, dtype=np.uint64).reshape(n, C.sizeof(_ffi.TileResult) // 8)
        rv[:, 0] = np.uint64(big.ctypes.data) + 8 * off[:-1].astype(np.uint64)
        return np.split(big, off[1:-1]), [], res

    def render_tasks(self, tasks, max_paths=0, tone_map=None, integrator=0, splats_out=None, splat_film=None,
                     max_vertices=0, sampler=0):
        """lumo_render_tiles over `tasks`; returns per-task (rgb_w array, result).
        tone_map: None, ToneMap.clamp(x) or ToneMap.REINHARD (tone_mapping.rs).
        sampler: SamplerType (samplers.rs:6-17; default MultiJittered).
        integrator = Integrator.BDPathTrace: the light-tracing splats of each task are appended
        to `splats_out` (a list of (x, y, rgb) record arrays, lumo's order), or, when
        `splats_out` is None, summed into `splat_film` (an H x W x 3 float64 array)."""
        L = lib()
        n = len(tasks)
        arr = tasks if isinstance(tasks, C.Array) else (_ffi.TileTask * n)(*tasks)
        tm = tone_map or ToneMap.NO_MAP
        lists = integrator == Integrator.BDPathTrace and splats_out is not None
        if integrator == Integrator.BDPathTrace and not lists:
            if splat_film is None or splat_film.dtype != np.float64 or not splat_film.flags.c_contiguous:
                raise ValueError("BDPT needs splats_out or a C-contiguous float64 splat_film")
        caps = None
        if lists:  # splat-list capacity per task: 16 taps per camera sample to start with
            tv = np.frombuffer(arr, dtype=np.uint64).reshape(n, C.sizeof(_ffi.TileTask) // 8)
            caps = (16 * (tv[:, 2] - tv[:, 0]) * (tv[:, 3] - tv[:, 1]) * tv[:, 5]).astype(np.int64).tolist()
        while True:
            bufs, sbufs, res = self._result_buffers(arr, n)
            if lists:
                for i in range(n):
                    sb = (_ffi.Splat * max(caps[i], 1))()
                    sbufs.append(sb)
                    res[i].splats = sb
                    res[i].splat_cap = caps[i]
            cfg = _ffi.RenderCfg(integrator, 0, max_paths, tm[0], tm[1], max_vertices, int(sampler),
                                 splat_film.ctypes.data_as(_ffi.c_double_p) if (splat_film is not None and not lists)
                                 else None)
            st = L.lumo_render_tiles(self.ctx, arr, n, C.byref(cfg), res)
            if st == _ffi.LUMO_ERR_OOM and lists and any(r.num_splats > c for r, c in zip(res, caps)):
                caps = [max(c, r.num_splats) for c, r in zip(caps, res)]  # splat lists too small: retry
                continue
            check(st, "render_tiles")
            break
        if lists:
            for i in range(n):
                m = res[i].num_splats
                a = (np.ctypeslib.as_array(sbufs[i])[:m] if m else
                     np.zeros(0, dtype=[("x", "<u4"), ("y", "<u4"), ("rgb", "<f8", (3,))]))
                splats_out.append(a.copy())
        return bufs, res

    def trace(self, origins, dirs, lights=None):
        """lumo_trace: closest hit (Scene::hit, scene.rs:119-147) of each ray, or with `lights`
        the visibility of that light (Scene::hit_light, scene.rs:165-189).  Returns t, kind
        (0 miss, 1 object, 2 light), object/light index, triangle index."""
        n = len(origins)
        o = np.ascontiguousarray(origins, dtype=np.float64).reshape(n, 3)
        d = np.ascontiguousarray(dirs, dtype=np.float64).reshape(n, 3)
        li = None if lights is None else np.ascontiguousarray(lights, dtype=np.int32)
        rays = _ffi.RaySoA(o.ctypes.data_as(_ffi.c_double_p), d.ctypes.data_as(_ffi.c_double_p), None,
                           None if li is None else li.ctypes.data_as(_ffi.c_int32_p))
        t = np.zeros(n)
        kind, obj, prim = (np.zeros(n, dtype=np.int32) for _ in range(3))
        hits = _ffi.HitSoA(t.ctypes.data_as(_ffi.c_double_p), kind.ctypes.data_as(_ffi.c_int32_p),
                           obj.ctypes.data_as(_ffi.c_int32_p), prim.ctypes.data_as(_ffi.c_int32_p))
        check(lib().lumo_trace(self.ctx, C.byref(rays), n, C.byref(hits), int(li is not None)), "trace")
        return t, kind, obj, prim

    def scene_info(self):
        """Kernel variant chosen for the uploaded scene (stack class, LDS bytes, feature class)."""
        s = _ffi.SceneInfo()
        check(lib().lumo_scene_info(self.ctx, C.byref(s)), "scene_info")
        return s

    def stats(self):
        s = _ffi.Stats()
        check(lib().lumo_stats_get(self.ctx, C.byref(s)), "stats")
        return s

    def busy_ms(self, stages):
        """Union of the timed launch intervals of `stages` (indices into _ffi.STAGES) since the
        last stats reset: the time at least one of them was running (lumo_stats_busy_ms)."""
        mask = 0
        for k in stages:
            mask |= 1 << int(k)
        ms = C.c_double(0.0)
        check(lib().lumo_stats_busy_ms(self.ctx, mask, C.byref(ms)), "stats_busy_ms")
        return ms.value

    def set_option(self, name, value):
        """lumo_set_option: one of _ffi.OPTIONS (LUMO_OPT_*); scheduling only, results unchanged."""
        check(lib().lumo_set_option(self.ctx, _ffi.OPT[name], int(value)), f"set_option({name}={value})")
        return self

    def option(self, name):
        v = C.c_int64(0)
        check(lib().lumo_get_option(self.ctx, _ffi.OPT[name], C.byref(v)), f"get_option({name})")
        return v.value

    def last_schedule(self):
        """lumo_last_schedule: the pass loop, streams, units, groups and merged passes of the last
        render_tasks call."""
        s = _ffi.ScheduleInfo()
        check(lib().lumo_last_schedule(self.ctx, C.byref(s)), "last_schedule")
        return s

    def close(self):
        if getattr(self, "ctx", None):
            lib().lumo_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Renderer:
    """Renderer::new(scene, camera) builder (renderer.rs:24-100); GPU tile dispatch."""

    def __init__(self, scene, camera):
        self.scene = scene.build()
        self.camera = camera
        self._samples = 1
        self._seed = None
        self._integrator = Integrator.PathTrace
        self._device = 0
        self._tone_map = ToneMap.NO_MAP
        self._sampler = SamplerType.MultiJittered

    def samples(self, n):
        self._samples = int(n)
        return self

    def seed(self, s):
        self._seed = int(s)
        return self

    def integrator(self, i):
        """Renderer::integrator (renderer.rs:72-75): PathTrace or BDPathTrace."""
        if i not in (Integrator.PathTrace, Integrator.BDPathTrace):
            raise ValueError(f"unknown integrator {i}")
        self._integrator = i
        return self

    def sampler(self, s):
        """Renderer::sampler (renderer.rs:89-93): a SamplerType."""
        if s not in (SamplerType.MultiJittered, SamplerType.Uniform, SamplerType.Jittered, SamplerType.Sobol):
            raise ValueError(f"unknown sampler {s}")
        self._sampler = s
        return self

    def tone_map(self, tm):
        """Renderer::tone_map (renderer.rs:66-69)."""
        self._tone_map = tm
        return self

    def device(self, d):
        self._device = int(d)
        return self

    def render(self, rank=0, world_size=1, schedule="static", chunk=None, store=None, key=None, timeout=None):
        """Render all (batch, tile) tasks and return this rank's (partial) film.

        With world_size > 1, `schedule="static"` renders the tiles with
        tile_index % world_size == rank; `schedule="dynamic"` claims
        chunks of `chunk` tiles from a `dist.TileQueue` in the process group's store until none
        are left (lumo's shared task receiver, pool.rs:26, 41-54), for scenes whose tiles cost
        unequal time.  Either way the reduced film is the single-process film.  `store` / `key` /
        `timeout` go to the TileQueue: with `key` the queue needs no process group, and `timeout`
        bounds the wait for the other ranks after this rank's last chunk (default: the store's
        timeout; dist.TileQueue)."""
        import time
        if schedule not in ("static", "dynamic"):
            raise ValueError(f"unknown schedule {schedule!r}")
        if self._seed is None:
            seed = [time.time_ns() & 0xFFFFFFFFFFFFFFFF or 1]
            if world_size > 1:  # every rank must render its tiles with the same task seeds
                import torch.distributed as dist
                if not dist.is_initialized():
                    raise ValueError("Renderer.render(rank, world_size > 1): set .seed() or initialise torch.distributed")
                dist.broadcast_object_list(seed, src=0)  # rank 0's seed
            self._seed = seed[0]
        w, h = self.camera.resolution
        tasks = make_tasks(w, h, self._samples, self._seed)
        from .dist import TileQueue, shard_tasks, tasks_of_tiles
        if schedule == "static" or world_size == 1:
            chunks = iter([shard_tasks(tasks, w, h, rank, world_size)])
        else:
            queue = TileQueue(w, h, world_size, chunk=chunk, store=store, key=key, timeout=timeout)
            chunks = (tasks_of_tiles(tasks, w, h, tiles) for tiles in queue)
        dev = Device(self._device)
        dev.upload(self.scene, self.camera)
        film = Film(w, h, getattr(self.camera, "color_space", 1), samples=self._samples)
        self.num_rays = self.num_camera_rays = 0
        self.tasks_rendered = 0
        for mine in chunks:
            if self._integrator == Integrator.BDPathTrace:
                # light-tracing splats are summed on the device straight into the film's splat buffer
                bufs, res = dev.render_tasks(mine, tone_map=self._tone_map, integrator=self._integrator,
                                             splat_film=film.splats, sampler=self._sampler)
            else:
                bufs, res = dev.render_tasks(mine, tone_map=self._tone_map, sampler=self._sampler)
            for t, b in zip(mine, bufs):
                film.add_tile(t, b)
            self.num_rays += sum(r.num_rays for r in res)
            self.num_camera_rays += sum(r.num_camera_rays for r in res)
            self.tasks_rendered += len(mine)
        dev.close()
        return film
