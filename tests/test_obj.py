""".obj / .mtl ingest (parser.rs, parser/obj.rs, parser/mtl.rs): tokenisation, negative indices,
normals/uvs, usemtl groups -> one mesh each, emissive groups -> Triangle lights, MTL -> material
parameters, zip members, and a render through the oracle."""
import math
import zipfile

import numpy as np
import pytest

import lumo_amd as L

MTL = b"""# two diffuse, a metal, a glass and a lamp
newmtl white
Kd 0.8 0.8 0.8
Ns 100
newmtl red
Kd 0.8 0.1 0.1
newmtl metal
Ks 0.9 0.9 0.9
Ns 400
Ni 1.5
illum 5
newmtl glass
Tf 1 1 1
Ni 1.5
Ns 900
illum 7
newmtl lamp
Ke 10 9 8
"""

OBJ = b"""# a floor, a box, a glass quad and a lamp quad
mtllib scene.mtl
v -2 0 -2
v  2 0 -2
v  2 0  2
v -2 0  2
vn 0 1 0
vn 0 0 0
vt 0 0
vt 1 0
vt 1 1
vt 0 1
g floor
usemtl white
f 1/1/1 4/4/1 3/3/1 2/2/1
v -0.5 0 -0.5
v  0.5 0 -0.5
v  0.5 1 -0.5
v -0.5 1 -0.5
o box
usemtl red
f -4 -1 -2 -3
usemtl metal
f 5 6 7
usemtl glass
f 5//2 7//2 8//2
v -0.3 2 -0.3
v  0.3 2 -0.3
v  0.3 2  0.3
v -0.3 2  0.3
usemtl lamp
f -4 -3 -2 -1
"""


def test_scene_from_obj_and_mtl(tmp_path):
    (tmp_path / "scene.obj").write_bytes(OBJ)
    (tmp_path / "scene.mtl").write_bytes(MTL)
    s = L.Scene.from_file(str(tmp_path / "scene.obj"), mtllib=str(tmp_path / "scene.mtl"))
    d = s.desc()
    assert d.num_objects == 4          # white, red, metal, glass groups
    assert d.num_lights == 2           # the lamp quad -> two Triangle lights
    assert all(d.lights[i].type == 2 for i in range(2))
    mats = [d.materials[i] for i in range(d.num_materials)]
    kinds = sorted(m.kind for m in mats)
    assert kinds == [2, 3, 3, 4, 5]    # light, 2x MfDiffuse, conductor, dielectric
    by_kind = {m.kind: m for m in mats}
    assert by_kind[4].roughness == pytest.approx(1.0 - math.sqrt(400) / 30.0)
    assert by_kind[5].roughness == pytest.approx(1e-5)  # Ns 900 -> 0 -> max(0, 1e-5)
    assert by_kind[5].eta_idx == 9      # transparent eta 1.5 -> glass dispersion curve
    # shading normals and uvs survive for the floor, the degenerate normal becomes +Z
    assert d.num_normals >= 2 and d.num_uvs == 4
    nrm = np.ctypeslib.as_array(d.normals, shape=(d.num_normals * 3,)).reshape(-1, 3)
    assert any(np.allclose(n, [0, 0, 1]) for n in nrm)


def test_zip_member_and_render(tmp_path):
    z = tmp_path / "scene.zip"
    with zipfile.ZipFile(z, "w") as f:
        f.writestr("Scene/scene.obj", OBJ)
        f.writestr("Scene/scene.mtl", MTL)
    s = L.Scene.from_file(str(z), "scene.obj", "scene.mtl")
    import oracle_ffi as O
    cam = L.Camera.builder().origin(0.0, 1.2, 4.0).towards(0.0, 0.5, 0.0).resolution((24, 16)).build()
    tasks = L.make_tasks(24, 16, 4, 3)
    bufs, res, _ = O.render_tasks(s.desc(), cam.desc, tasks, O.WAVEFRONT, 4)
    f = L.Film(24, 16)
    for t, b in zip(tasks, bufs):
        f.add_tile(t, b)
    assert np.isfinite(f.rgb()).all() and f.rgb().mean() > 0


def test_mesh_from_obj_with_instance(tmp_path):
    s = L.Scene()
    ref = s.add_obj(OBJ, L.Material.diffuse(L.Spectrum.from_rgb(0.5, 0.5, 0.5)))
    ref.to_unit_size().to_origin()
    s.add_rectangle((-1e4, 1e4, -1e4), (-1e4 + 1, 1e4, -1e4), (-1e4 + 1, 1e4, -1e4 + 1),
                    L.Material.light(L.Spectrum.from_rgb(1, 1, 1)), light=True)
    d = s.desc()
    assert d.num_objects == 1 and d.objects[0].xform == 0
    assert d.objects[0].num_tris == 2 + 2 + 1 + 1 + 2  # every face in one mesh (usemtl ignored)


@pytest.mark.parametrize("bad", [b"v 1 2\n", b"v 0 0 0\nf 1 2 3\n", b"usemtl nope\nf 1 2 3\n"])
def test_obj_errors(bad):
    with pytest.raises(ValueError):
        L.Scene.from_file(_tmp_obj(bad))


def _tmp_obj(data):
    import tempfile
    f = tempfile.NamedTemporaryFile(suffix=".obj", delete=False)
    f.write(data)
    f.close()
    return f.name


def test_texture_map_missing_file():
    """parser.rs:_extract_zip: a map_Kd naming a file the archive lacks is an error."""
    mtl = b"newmtl t\nKd 1 1 1\nmap_Kd wall.png\n"
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        open(d + "/a.obj", "wb").write(b"v 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl t\nf 1 2 3\n")
        open(d + "/a.mtl", "wb").write(mtl)
        with pytest.raises(ValueError, match="wall.png"):
            L.Scene.from_file(d + "/a.obj", mtllib=d + "/a.mtl")


def test_plain_files_register_only_named_textures(tmp_path):
    """Scene.from_file on plain files: the MTL's map_Kd name resolves by _extract_zip's
    case-insensitive suffix rule under the MTL's directory (parser.rs:88-114); only named files are
    read, an unrelated unreadable file is ignored, and a name two files match is reported as
    ambiguous ("Found multiple"), not as missing."""
    import numpy as np_
    from imgdata import random_png
    png = random_png(np_.random.default_rng(1), 4, 4, 2, 8)[0]
    mtl = MTL.replace(b"newmtl red\n", b"newmtl red\nmap_Kd tex/Red.PNG\n")
    (tmp_path / "scene.obj").write_bytes(OBJ)
    (tmp_path / "scene.mtl").write_bytes(mtl)
    (tmp_path / "tex").mkdir()
    (tmp_path / "tex" / "red.png").write_bytes(png)
    (tmp_path / "unrelated.png").mkdir()  # a directory with an image's name: never opened
    s = L.Scene.from_file(str(tmp_path / "scene.obj"), mtllib=str(tmp_path / "scene.mtl"))
    assert s.desc().num_textures >= 1
    (tmp_path / "more").mkdir()
    (tmp_path / "more" / "tex").mkdir()
    (tmp_path / "more" / "tex" / "red.png").write_bytes(png)
    with pytest.raises(ValueError, match="several files match"):
        L.Scene.from_file(str(tmp_path / "scene.obj"), mtllib=str(tmp_path / "scene.mtl"))
    (tmp_path / "scene.mtl").write_bytes(MTL.replace(b"newmtl red\n", b"newmtl red\nmap_Kd nowhere.png\n"))
    with pytest.raises(ValueError, match="no file"):
        L.Scene.from_file(str(tmp_path / "scene.obj"), mtllib=str(tmp_path / "scene.mtl"))
