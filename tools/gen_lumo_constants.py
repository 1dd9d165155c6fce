#!/usr/bin/env python3
"""Extract the numeric constants of lumo's scene / camera / colour code that the product's host
side restates, as DATA, into tests/golden/lumo_constants.json (run at development time; needs
/root/reference; the JSON is committed and read by tests/test_constants.py):

* src/tracer/scene/cornell_box.rs:8-193: the five spectra point lists, the light rectangle and the
  seven meshes' vertices in lumo's order (with the face scheme: quads (0,1,2),(0,2,3); boxes five
  such quads), and each mesh's spectrum;
* src/tracer/camera.rs:139-148 (Camera::cornell_box) and camera/builder.rs:35-51 (defaults);
* src/tracer/camera/matrices.rs:3-13 (near / far of the perspective projection);
* src/tracer/color/space.rs:51-94 (primaries of sRGB / DCI-P3, the XYZ->LMS matrix);
* src/tracer/color/xyz.rs:34 (Y_INTEGRAL) and samples.rs (CIE 1931 X/Y/Z, illuminants D65 and
  CORNELL, 95 bins), color.rs:56-57 (LAMBDA_MIN / MAX), dense_spectrum.rs:5 (DENSE_SAMPLES);
* src/tracer/filter.rs:20-24 (default Gaussian radius / sigma = r / 4).
Numbers are parsed from the Rust literals with Python's float(), which rounds decimal literals
exactly as rustc does.
"""
import json
import os
import re
import sys

REF = "/root/reference/src"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden", "lumo_constants.json")
NUM = r"-?\d+(?:\.\d*)?(?:e-?\d+)?"


def read(rel):
    with open(os.path.join(REF, rel)) as f:
        return f.read()


def vec3s(text):
    return [[float(x) for x in m.group(1).split(",")] for m in re.finditer(r"Vec3::new\(([^)]*)\)", text)]


def cornell():
    src = read("tracer/scene/cornell_box.rs")
    spectra = {m.group(1): m.group(2) for m in re.finditer(r"let (\w+)_spec = Spectrum::from_pts\(\"([^\"]*)\"\)", src)}
    # material bindings: `let floor = material(white_spec.clone());`
    mats = {m.group(1): m.group(2) for m in re.finditer(r"let (\w+) = material\((\w+)_spec", src)}
    blocks = list(re.finditer(r"/\* ([\w ]+) \*/", src))
    meshes = []
    light = None
    for k, b in enumerate(blocks):
        end = blocks[k + 1].start() if k + 1 < len(blocks) else len(src)
        body = src[b.end():end]
        name = b.group(1).strip()
        v = vec3s(body)
        if name == "light":
            light = v
            continue
        m = re.search(r"add_object\(vertices, (\w+), (None|Some\(box_faces\(\)\))\)", body)
        meshes.append({"name": name, "vertices": v, "material": m.group(1),
                       "faces": "quad" if m.group(2) == "None" else "box"})
    for me in meshes:
        me["spectrum"] = mats[me["material"]]
    light_spec = re.search(r"Material::Light\(\s*Texture::from\((\w+)_spec\),\s*illuminants::(\w+),\s*(" + NUM +
                           r"),\s*(true|false)", src)
    return {"spectra": spectra, "light_vertices": light, "meshes": meshes,
            "light": {"spectrum": light_spec.group(1), "illuminant": light_spec.group(2),
                      "scale": float(light_spec.group(3)), "two_sided": light_spec.group(4) == "true"}}


def call_args(text, name):
    m = re.search(r"\." + name + r"\(([^)]*)\)", text)
    return [float(x) for x in m.group(1).replace("(", "").split(",")]


def camera():
    src = read("tracer/camera.rs")
    fn = src[src.index("pub fn cornell_box() -> Camera"):]
    fn = fn[:fn.index("}")]
    cb = {"origin": call_args(fn, "origin"), "towards": call_args(fn, "towards"), "zoom": call_args(fn, "zoom")[0],
          "focal_length": call_args(fn, "focal_length")[0], "resolution": call_args(fn, "resolution"),
          "illuminant": re.search(r"illuminants::(\w+)", fn).group(1)}
    b = read("tracer/camera/builder.rs")
    nb = b[b.index("pub fn new() -> Self"):]
    nb = nb[:nb.index("}\n")]
    defaults = {"zoom": float(re.search(r"zoom: (" + NUM + ")", nb).group(1)),
                "lens_radius": float(re.search(r"lens_radius: (" + NUM + ")", nb).group(1)),
                "focal_length": float(re.search(r"focal_length: (" + NUM + ")", nb).group(1)),
                "vfov": float(re.search(r"vfov: (" + NUM + ")", nb).group(1)),
                "resolution": [float(x) for x in re.search(r"resolution: \((\d+), (\d+)\)", nb).groups()],
                "origin": "ZERO" if "origin: Point::ZERO" in nb else None,
                "towards": "-Z" if "towards: -Point::Z" in nb else None,
                "up": "Y" if "up: Direction::Y" in nb else None,
                "illuminant": re.search(r"illuminant: illuminants::(\w+)", nb).group(1)}
    mt = read("tracer/camera/matrices.rs")
    pp = mt[mt.index("pub fn perspective_projection"):mt.index("pub fn orthographic_projection")]
    proj = {"near": float(re.search(r"let near = (" + NUM + ")", pp).group(1)),
            "far": float(re.search(r"let far = (" + NUM + ")", pp).group(1))}
    return {"cornell_box": cb, "defaults": defaults, "perspective": proj}


def colour():
    sp = read("tracer/color/space.rs")
    prim = {}
    for name in ("sRGB", "DCI_P3"):
        m = re.search(name + r"_XYZ_to_RGB: Mat3 = Self::xyz_to_rgb\(([^;]*)\);", sp)
        prim[name] = [[float(a), float(b)] for a, b in re.findall(r"Vec2::new\((" + NUM + r"), (" + NUM + r")\)",
                                                                 m.group(1))]
    lms = re.search(r"XYZ_to_LMS: Mat3 = Mat3::new\(([^;]*)\);", sp).group(1)
    lms_rows = [[float(x) for x in re.findall(NUM, r)] for r in re.findall(r"Vec3::new\(([^)]*)\)", lms)]
    default_cs = re.search(r"pub fn default\(\) -> &'static Self \{\s*&Self::(\w+)", sp).group(1)
    xyz = read("tracer/color/xyz.rs")
    y_int = float(re.search(r"Y_INTEGRAL: Float = (" + NUM + ")", xyz).group(1))
    samples = read("tracer/color/samples.rs")
    tables, group = {}, None
    for m in re.finditer(r"pub mod (\w+)\s*\{|(\w+),\s*\[([^\]]*)\]", samples):
        if m.group(1):
            group = m.group(1)
            continue
        toks = [t for t in re.split(r"[\s,]+", m.group(3)) if t]
        tables[f"{group}.{m.group(2)}"] = [float(t) for t in toks]
    keep = {k: tables[k] for k in ("cie1931.X", "cie1931.Y", "cie1931.Z", "illuminants.D65", "illuminants.CORNELL")}
    cr = read("tracer/color.rs")
    ds = read("tracer/color/dense_spectrum.rs")
    lam = {"min": float(re.search(r"LAMBDA_MIN: Float = (" + NUM + ")", cr).group(1)),
           "max": float(re.search(r"LAMBDA_MAX: Float = (" + NUM + ")", cr).group(1)),
           "samples": int(re.search(r"DENSE_SAMPLES: usize = (\d+)", ds).group(1))}
    return {"primaries": prim, "xyz_to_lms": lms_rows, "default_color_space": default_cs, "y_integral": y_int,
            "tables": keep, "lambda": lam}


def filt():
    f = read("tracer/filter.rs")
    m = re.search(r"fn default\(\) -> Self \{\s*Self::gaussian\((" + NUM + r"), (" + NUM + r") / (" + NUM + r")\)", f)
    return {"gaussian_radius": float(m.group(1)), "gaussian_sigma": float(m.group(2)) / float(m.group(3))}


def main():
    out = {"source": "ekarpp/lumo v0.6.1 via tools/gen_lumo_constants.py (numeric literals only)",
           "cornell": cornell(), "camera": camera(), "colour": colour(), "filter": filt()}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    sys.exit(main())
