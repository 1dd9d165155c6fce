"""lumo's example scenes used by the benchmark configurations (BASELINE.json configs), built
through the same builder API a lumo user calls.  Downloaded assets are replaced by the
procedural stand-ins of lumo_amd.procedural."""
import math

from . import Camera, Material, Scene, Spectrum, named_spectrum
from .procedural import dragon_standin, suzanne_standin


def cornell():
    """examples/cornell.rs: Scene::cornell_box + Camera::cornell_box."""
    return Scene.cornell_box()


def dragon(mesh=None):
    """examples/dragon.rs:6-35 with the dragon .obj replaced by `mesh` (vertices, faces);
    default: the 871 414-triangle procedural stand-in."""
    v, f = mesh if mesh is not None else dragon_standin()
    scene = Scene.empty_box(Spectrum.from_srgb(242, 242, 242), Material.diffuse(named_spectrum("RED")),
                            Material.diffuse(named_spectrum("GREEN")))
    scene.add_mesh(v, f, Material.transparent(named_spectrum("MAGENTA"), 0.03, 1.5)) \
        .to_unit_size().to_origin().rotate_y(5.0 * math.pi / 8.0).scale_uniform(1.3).set_y(-0.799) \
        .translate(0.0, 0.0, -1.4)
    return scene


def default_camera(resolution):
    """Camera::builder().build() with the resolution overridden."""
    return Camera.builder().resolution(resolution).build()


def bistro(standin=None):
    """Bistro exterior (examples/bistro.rs, night variant) as a procedural stand-in: every
    material group is its own mesh, emissive faces are Triangle lights, plus a constant
    environment light (the HDR map is not available)."""
    from . import Material, Spectrum
    from .procedural import bistro_standin
    groups, lamps = standin if standin is not None else bistro_standin()
    scene = Scene()
    for v, f, kind, rgb in groups:
        spec = Spectrum.from_rgb(*rgb)
        mat = Material.metal(spec, 0.25, 1.5, 3.0) if kind == "metal" else Material.diffuse(spec)
        scene.add_mesh(v, f, mat)
    # D65 / Light emission is ~100 x the texture (dense illuminant scale), like bistro.rs's 0.001 HDR scale
    lamp_mat = Material.light(Spectrum.from_srgb(255, 197, 143), scale=0.5)
    for v, f in lamps:
        scene.add_mesh(v, f, lamp_mat, light=True)
    scene.set_environment_map(Spectrum.from_rgb(0.3, 0.4, 0.8), 0.002)
    return scene


def bistro_camera(resolution):
    """bistro.rs:15-18 exterior camera."""
    return Camera.builder().origin(-16.0, 5.0, -1.0).towards(0.0, 0.0, 0.0).resolution(resolution).build()


def caustics(mesh=None):
    """examples/caustics.rs:7-37: empty box with MAGENTA / CYAN walls, a mirror and a glass copy
    of suzanne (`mesh` = (vertices, faces); default: the 968-triangle procedural stand-in),
    each to_unit_size -> to_origin -> rotations -> translate."""
    v, f = mesh if mesh is not None else suzanne_standin()
    scene = Scene.empty_box(Spectrum.from_srgb(242, 242, 242), Material.diffuse(named_spectrum("MAGENTA")),
                            Material.diffuse(named_spectrum("CYAN")))
    pi = math.pi
    scene.add_mesh(v, f, Material.mirror()).to_unit_size().to_origin() \
        .rotate_y(-pi / 8.0).rotate_z(pi / 8.0).rotate_x(-pi / 8.0).translate(0.5, -0.3, -1.0)
    scene.add_mesh(v, f, Material.glass()).to_unit_size().to_origin() \
        .rotate_y(pi / 8.0).rotate_z(-pi / 8.0).rotate_x(pi / 16.0).translate(-0.35, 0.25, -1.25)
    return scene


def caustics_camera(resolution):
    """caustics.rs:7-10: origin (0, 0, 2), zoom 3."""
    return Camera.builder().origin(0.0, 0.0, 2.0).zoom(3.0).resolution(resolution).build()
