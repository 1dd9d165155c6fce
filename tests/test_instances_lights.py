"""Instances (object/instance.rs) and triangle lights (triangle.rs Sampleable, parser/obj.rs
emissive faces) in the host builder and the oracle: lumo's kd `intersects` test with the real
to_unit_size().to_origin() instance chain, transformed bounds, the test_util.rs
`sampled_rays_hit` property and solid-angle normalisation of the light pdfs."""
import math

import numpy as np
import pytest

import lumo_amd as L
import oracle_ffi as O
from lumo_amd import named_spectrum as NS
from test_host import CUBE_F, CUBE_V, tiny_light
from test_oracle import sphere_points


def grey():
    return L.Material.lambertian(L.Spectrum.from_rgb(0.5, 0.5, 0.5))


def test_kd_intersects_instanced_unit_cube():
    """kdtree_tests.rs:52-80 with the mesh wrapped as in the test: to_unit_size().to_origin()."""
    s = L.Scene()
    s.add_mesh(np.array(CUBE_V, dtype=float), CUBE_F, grey()).to_unit_size().to_origin()
    tiny_light(s)
    d = s.desc()
    assert d.num_transforms == 1 and d.objects[0].xform == 0
    b = d.object_nodes[0]
    np.testing.assert_allclose(np.array(b.bmax[:]) + np.array(b.bmin[:]), 0.0, atol=1e-12)
    assert max(np.array(b.bmax[:]) - np.array(b.bmin[:])) == pytest.approx(1.0)
    xo = sphere_points(10000, 3, 5.0)
    xo = xo[xo[:, 1] > -0.1]  # open bottom
    dr = -xo / np.linalg.norm(xo, axis=1, keepdims=True)
    t, kind, obj, _ = O.trace(d, xo, dr)
    assert np.all(kind == 1) and np.all((t > 4.0) & (t < 5.0))


def test_instance_equals_pretransformed_mesh():
    """A rotated / scaled / translated instance is hit where the explicitly transformed mesh is."""
    v = np.array(CUBE_V, dtype=float)
    a = L.Scene()
    a.add_mesh(v, CUBE_F, grey()).rotate_y(5 * math.pi / 8).scale_uniform(0.01).translate(0.3, -0.2, 0.5)
    tiny_light(a)
    c, s_ = math.cos(5 * math.pi / 8), math.sin(5 * math.pi / 8)
    R = np.array([[c, 0, s_], [0, 1, 0], [-s_, 0, c]])
    vb = (v @ R.T) * 0.01 + np.array([0.3, -0.2, 0.5])
    b = L.Scene()
    b.add_mesh(vb, CUBE_F, grey())
    tiny_light(b)
    rng = np.random.default_rng(5)
    o = rng.normal(size=(4000, 3)) * 3
    tgt = np.array([0.3, 1.0, 0.5]) * np.array([1, 0, 1]) + rng.uniform(-1, 1, (4000, 3)) * np.array([1.2, 1.6, 1.2])
    dr = tgt - o
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    ta, ka, _, _ = O.trace(a.desc(), o, dr)
    tb, kb, _, _ = O.trace(b.desc(), o, dr)
    agree = ka == kb
    assert agree.mean() > 0.999
    both = agree & (ka == 1)
    assert both.sum() > 200
    np.testing.assert_allclose(ta[both], tb[both], rtol=1e-9)


def test_instance_ops_validate():
    s = L.Scene()
    r = s.add_mesh(np.array(CUBE_V, dtype=float), CUBE_F, grey())
    with pytest.raises(Exception):
        r.scale(0.0, 1.0, 1.0)
    r.translate(1, 2, 3)
    with pytest.raises(Exception):
        r.to_unit_size()  # only on the kd-tree itself (kdtree.rs:93-99)


def quad(y, half, flip=False):
    v = np.array([(-half, y, -half), (half, y, -half), (half, y, half), (-half, y, half)], dtype=float)
    f = [(0, 1, 2, 3)] if not flip else [(0, 3, 2, 1)]  # default winding: normal -y (emits downwards)
    return v, f


def light_scene(kind):
    s = L.Scene()
    white = NS("WHITE")
    if kind == "triangles":
        v, f = quad(2.0, 0.5)
        s.add_mesh(v, f, L.Material.light(white), light=True)
    elif kind == "instanced_rect":
        s.add_rectangle((-0.25, 0.0, -0.25), (0.25, 0.0, -0.25), (0.25, 0.0, 0.25), L.Material.light(white),
                        light=True).rotate_y(0.3).scale_uniform(2.0).translate(0.1, 2.0, -0.2)
    elif kind == "tilted_rect":
        s.add_rectangle((-0.25, 0.0, -0.25), (0.25, 0.0, -0.25), (0.25, 0.0, 0.25), L.Material.light(white),
                        light=True).rotate_x(0.3).scale_uniform(2.0).translate(0.1, 2.0, -0.2)
    else:
        s.add_rectangle((-0.5, 2.0, -0.5), (0.5, 2.0, -0.5), (0.5, 2.0, 0.5), L.Material.light(white), light=True)
    s.add_rectangle((-3, -1, -3), (3, -1, -3), (3, -1, 3), grey())
    return s


@pytest.mark.parametrize("kind", ["triangles", "instanced_rect", "tilted_rect", "rect"])
def test_sampled_light_rays_hit(kind):
    """test_util.rs:59-75 sampled_rays_hit: every sample_towards direction hits the light and
    has positive pdf."""
    s = light_scene(kind)
    d = s.desc()
    xo = np.array([0.2, -0.5, 0.1])
    for li in range(d.num_lights):
        wi = O.light_sample(d, li, xo, 4000, 11 + li)
        pdf = O.light_pdf(d, li, xo, wi)
        assert np.all(pdf > 0), (kind, li, np.mean(pdf > 0))


@pytest.mark.parametrize("kind", ["triangles", "instanced_rect", "rect"])
def test_light_pdf_normalised(kind):
    """The solid-angle pdf integrates to 1 over the directions that hit the light:
    E_{w ~ uniform sphere}[4 pi pdf(w)] = 1."""
    s = light_scene(kind)
    d = s.desc()
    xo = np.array([0.2, -0.5, 0.1])
    rng = np.random.default_rng(2)
    w = rng.normal(size=(400000, 3))
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    w[:, 1] = np.abs(w[:, 1])  # the lights are above xo
    for li in range(d.num_lights):
        pdf = O.light_pdf(d, li, xo, w)
        est = 2 * np.pi * pdf.mean()
        assert est == pytest.approx(1.0, abs=0.03), (kind, li, est)


def test_triangle_lights_split_mesh():
    s = light_scene("triangles")
    d = s.desc()
    assert d.num_lights == 2
    assert all(d.lights[i].type == 2 and d.lights[i].kd_root == -1 for i in range(2))
    np.testing.assert_allclose([d.lights[i].area for i in range(2)], [0.5, 0.5])
    # alias table by power = area x emission -> uniform for equal halves
    np.testing.assert_allclose([d.alias_pdf[i] for i in range(2)], [0.5, 0.5], rtol=1e-12)


def test_light_scenes_render_the_same_expectation():
    """A quad light made of two Triangle lights and the same quad as a Rectangle light give the
    same image in expectation (n_shadow and light selection differ)."""
    cam = L.Camera.builder().origin(0.0, 0.5, 4.0).towards(0.0, -0.5, 0.0).resolution((32, 32)).build()
    means = {}
    for kind in ("triangles", "rect"):
        s = light_scene(kind)
        runs = []
        for seed in range(1, 7):
            tasks = L.make_tasks(32, 32, 16, seed)
            bufs, _, _ = O.render_tasks(s.desc(), cam.desc, tasks, O.WAVEFRONT, 8)
            f = L.Film(32, 32)
            for t, b in zip(tasks, bufs):
                f.add_tile(t, b)
            runs.append(np.nanmean(f.rgb(), axis=(0, 1)))
        means[kind] = np.array(runs)
    a, b = means["triangles"], means["rect"]
    se = np.sqrt(a.var(0, ddof=1) / len(a) + b.var(0, ddof=1) / len(b))
    z = np.abs(a.mean(0) - b.mean(0)) / np.maximum(se, 1e-12)
    assert np.all(z < 4.0), (a.mean(0), b.mean(0), z)


def test_tilted_instance_light_pdf_quirk():
    """instance.rs:170 maps the world normal to local space with normal_transform.inv().transpose()
    = M (not M^T), so for an instanced light rotated about an axis other than its normal the pdf
    is not normalised.  The restatement keeps lumo's formula: the integral differs from 1 by the
    same amount in the oracle and (bit-exactly) on the GPU."""
    s = light_scene("tilted_rect")
    d = s.desc()
    xo = np.array([0.2, -0.5, 0.1])
    rng = np.random.default_rng(2)
    w = rng.normal(size=(400000, 3))
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    w[:, 1] = np.abs(w[:, 1])
    est = 2 * np.pi * O.light_pdf(d, 0, xo, w).mean()
    assert abs(est - 1.0) > 0.05


def sphere_scene(env=False, light_sphere=True):
    s = L.Scene()
    if light_sphere:
        s.add_sphere(0.3, L.Material.light(NS("WHITE")), light=True).translate(0.0, 1.5, 0.0)
    s.add_sphere(0.5, L.Material.diffuse(L.Spectrum.from_rgb(0.7, 0.6, 0.5)))
    s.add_rectangle((-3, -1, -3), (3, -1, -3), (3, -1, 3), grey())
    if env:
        s.set_environment_map(L.Spectrum.from_rgb(0.4, 0.5, 0.9), 0.5)
    return s


def test_sphere_intersections():
    """test_util.rs object tests on Sphere::new(1.0): no self-intersection from the surface,
    nothing behind, hits towards the centre; hit_t agrees with hit (shadow_hit_accurate)."""
    s = L.Scene()
    s.add_sphere(1.0, grey())
    tiny_light(s)
    d = s.desc()
    t, k, _, _ = O.trace(d, np.array([(1.0 + 1e-10, 0, 0), (2.0, 0, 0)]), np.array([(0, 0, 1.0), (1.0, 0, 0)]))
    assert np.all(k == 0)
    p = np.array([1.23, 4.56, 7.89])
    t, k, _, _ = O.trace(d, p[None], -p[None] / np.linalg.norm(p))
    assert k[0] == 1 and t[0] == pytest.approx(np.linalg.norm(p) - 1.0)
    xo = sphere_points(5000, 9, 5.0)
    t, k, _, _ = O.trace(d, xo, -xo / 5.0)
    assert np.all(k == 1) and np.allclose(t, 4.0)


@pytest.mark.parametrize("where", [(0.2, -0.5, 0.1), (0.0, 1.55, 0.05)])
def test_sphere_light_sampling(where):
    """sampled_rays_hit + pdf normalisation for a sphere light seen from outside (cone sampling)
    and from inside (area sampling)."""
    s = sphere_scene()
    d = s.desc()
    xo = np.array(where)
    wi = O.light_sample(d, 0, xo, 4000, 3)
    assert np.all(O.light_pdf(d, 0, xo, wi) > 0)
    rng = np.random.default_rng(4)
    w = rng.normal(size=(2000000, 3))  # the outside case subtends ~0.6% of the sphere of directions
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    est = 4 * np.pi * O.light_pdf(d, 0, xo, w).mean()
    assert est == pytest.approx(1.0, abs=0.04)


def test_environment_map_sphere():
    """Scene::build adds a two-sided D65 Light sphere enclosing the scene bounds."""
    s = sphere_scene(env=True)
    d = s.desc()
    assert d.num_lights == 2
    env = d.lights[1]
    assert env.type == 3 and env.xform >= 0
    m = d.materials[env.material]
    assert m.kind == 2 and m.two_sided == 1 and m.scale == 0.5
    # a ray escaping the scene hits the environment from inside
    t, k, o, _ = O.trace(d, np.array([(0.0, 0.0, 2.0)]), np.array([(0.0, 0.0, 1.0)]))
    assert k[0] == 2 and o[0] == 1
    cam = L.Camera.builder().origin(0.0, 0.3, 4.0).towards(0.0, 0.0, 0.0).resolution((16, 16)).build()
    tasks = L.make_tasks(16, 16, 8, 5)
    bufs, _, _ = O.render_tasks(d, cam.desc, tasks, O.WAVEFRONT, 4)
    f = L.Film(16, 16)
    for tk, b in zip(tasks, bufs):
        f.add_tile(tk, b)
    img = f.rgb()
    assert np.all(np.isfinite(img)) and img[..., 2].mean() > img[..., 0].mean()  # bluish sky
