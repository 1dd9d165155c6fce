"""ctypes mirror of include/lumo_amd.h and include/lumo_host.h (the C-ABI boundary).

Only plain C types cross the boundary; no torch types.  `load()` loads the in-tree
liblumo_amd.so built by `make` (or __graft_entry__.build()).  The product raises if the
library is missing: there is no CPU fallback.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
ABI_VERSION = 10  # include/lumo_amd.h LUMO_ABI_VERSION
LIB_PATH = os.environ.get("LUMO_AMD_LIB") or os.path.join(_HERE, "liblumo_amd.so")

c_double_p = C.POINTER(C.c_double)
c_int32_p = C.POINTER(C.c_int32)
c_int64_p = C.POINTER(C.c_int64)
c_uint64_p = C.POINTER(C.c_uint64)
c_uint32_p = C.POINTER(C.c_uint32)

LUMO_OK = 0
LUMO_ERR_OOM = 7
STATUS = {0: "OK", 1: "INVALID", 2: "NO_DEVICE", 3: "HIP", 4: "NO_SCENE", 5: "NO_CAMERA",
          6: "UNSUPPORTED", 7: "OOM"}


class Spectrum(C.Structure):
    _fields_ = [("c0", C.c_float), ("c1", C.c_float), ("c2", C.c_float), ("scale", C.c_float)]


class Material(C.Structure):
    _fields_ = [("kind", C.c_int32), ("two_sided", C.c_int32), ("illuminant", C.c_int32),
                ("eta_idx", C.c_int32), ("k_idx", C.c_int32), ("flags", C.c_int32),
                ("scale", C.c_double), ("roughness", C.c_double),
                ("albedo", Spectrum), ("ks", Spectrum), ("tf", Spectrum),
                ("albedo_tex", C.c_int32), ("ks_tex", C.c_int32), ("tf_tex", C.c_int32), ("normal_map", C.c_int32)]


MAT_BLANK, MAT_LAMBERTIAN, MAT_LIGHT, MAT_MF_DIFFUSE, MAT_MF_CONDUCTOR, MAT_MF_DIELECTRIC = range(6)
TEX_SOLID, TEX_IMAGE, TEX_CHECKERBOARD, TEX_MARBLE, TEX_MANDELBROT = range(5)


class Texture(C.Structure):
    _fields_ = [("kind", C.c_int32), ("width", C.c_int32), ("height", C.c_int32), ("first", C.c_int32),
                ("second", C.c_int32), ("pad0", C.c_int32), ("scale", C.c_double), ("spec", Spectrum)]


class NormalMap(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("first", C.c_int32), ("pad0", C.c_int32)]


class Perlin(C.Structure):
    _fields_ = [("lattice", (C.c_double * 3) * 256), ("perm", (C.c_int32 * 256) * 3)]


class BvhNode(C.Structure):
    _fields_ = [("bmin", C.c_double * 3), ("bmax", C.c_double * 3), ("right", C.c_int32),
                ("first", C.c_int32), ("count", C.c_int32), ("pad0", C.c_int32)]


class KdNode(C.Structure):
    _fields_ = [("point", C.c_double), ("axis", C.c_int32), ("right", C.c_int32), ("leaf", C.c_int32),
                ("first", C.c_int32), ("count", C.c_int32), ("pad0", C.c_int32)]


class Transform(C.Structure):
    _fields_ = [("m", C.c_double * 16), ("inv", C.c_double * 16), ("nrm", C.c_double * 9), ("pad0", C.c_double)]


class Object(C.Structure):
    _fields_ = [("type", C.c_int32), ("material", C.c_int32), ("kd_root", C.c_int32), ("tri_base", C.c_int32),
                ("item_base", C.c_int32), ("num_tris", C.c_int32), ("xform", C.c_int32),
                ("material_override", C.c_int32), ("bmin", C.c_double * 3),
                ("bmax", C.c_double * 3), ("origin", C.c_double * 3), ("b0", C.c_double * 3),
                ("b1", C.c_double * 3), ("area", C.c_double), ("radius", C.c_double)]


class Triangle(C.Structure):
    _fields_ = [("v", C.c_int32 * 3), ("n", C.c_int32 * 3), ("t", C.c_int32 * 3), ("material", C.c_int32)]


class SceneDesc(C.Structure):
    _fields_ = [
        ("num_vertices", C.c_int32), ("num_normals", C.c_int32), ("num_uvs", C.c_int32),
        ("num_triangles", C.c_int32),
        ("vertices", c_double_p), ("normals", c_double_p), ("uvs", c_double_p),
        ("triangles", C.POINTER(Triangle)),
        ("num_kd_nodes", C.c_int32), ("num_kd_items", C.c_int32),
        ("kd_nodes", C.POINTER(KdNode)), ("kd_items", c_int32_p),
        ("num_objects", C.c_int32), ("num_object_nodes", C.c_int32), ("num_object_items", C.c_int32),
        ("objects", C.POINTER(Object)), ("object_nodes", C.POINTER(BvhNode)), ("object_items", c_int32_p),
        ("num_lights", C.c_int32), ("num_light_nodes", C.c_int32), ("num_light_items", C.c_int32),
        ("lights", C.POINTER(Object)), ("light_nodes", C.POINTER(BvhNode)), ("light_items", c_int32_p),
        ("alias_prob", c_double_p), ("alias_idx", c_int32_p), ("alias_pdf", c_double_p),
        ("num_materials", C.c_int32), ("num_dense_spectra", C.c_int32),
        ("materials", C.POINTER(Material)), ("dense_spectra", c_double_p),
        ("num_transforms", C.c_int32), ("pad1", C.c_int32), ("transforms", C.POINTER(Transform)),
        ("num_textures", C.c_int32), ("num_texels", C.c_int32),
        ("textures", C.POINTER(Texture)), ("texels", C.POINTER(Spectrum)),
        ("num_normal_maps", C.c_int32), ("num_normal_texels", C.c_int32),
        ("normal_maps", C.POINTER(NormalMap)), ("normal_texels", c_double_p),
        ("num_perlin", C.c_int32), ("pad2", C.c_int32), ("perlin", C.POINTER(Perlin)),
    ]


class CameraDesc(C.Structure):
    _fields_ = [
        ("world_to_camera", (C.c_double * 16) * 2), ("screen_to_raster", (C.c_double * 16) * 2),
        ("camera_to_screen", (C.c_double * 16) * 2),
        ("lens_radius", C.c_double), ("focal_length", C.c_double),
        ("width", C.c_int64), ("height", C.c_int64),
        ("orthographic", C.c_int32), ("illuminant", C.c_int32),
        ("white_balance", C.c_double * 9), ("xyz_to_rgb", C.c_double * 9),
        ("filter_radius", C.c_double), ("filter_sigma", C.c_double),
    ]


class TileTask(C.Structure):
    _fields_ = [("px_min", C.c_uint64 * 2), ("px_max", C.c_uint64 * 2), ("batch", C.c_uint64),
                ("samples", C.c_uint64), ("total_samples", C.c_uint64), ("seed", C.c_uint64)]


class Splat(C.Structure):
    _fields_ = [("x", C.c_uint32), ("y", C.c_uint32), ("rgb", C.c_double * 3)]


class TileResult(C.Structure):
    _fields_ = [("rgb_w", c_double_p), ("num_camera_rays", C.c_uint64), ("num_rays", C.c_uint64),
                ("num_queries", C.c_uint64), ("splats", C.POINTER(Splat)), ("splat_cap", C.c_uint64),
                ("num_splats", C.c_uint64)]


class RenderCfg(C.Structure):
    _fields_ = [("integrator", C.c_int32), ("rng_mode", C.c_int32), ("max_paths", C.c_int32),
                ("tone_map", C.c_int32), ("tone_arg", C.c_double), ("max_vertices", C.c_int32),
                ("sampler", C.c_int32), ("splat_film", c_double_p)]


class RaySoA(C.Structure):
    _fields_ = [("origin", c_double_p), ("dir", c_double_p), ("t_max", c_double_p), ("light", c_int32_p)]


class HitSoA(C.Structure):
    _fields_ = [("t", c_double_p), ("kind", c_int32_p), ("object", c_int32_p), ("prim", c_int32_p)]


class SceneInfo(C.Structure):
    _fields_ = [("stack_class", C.c_int32), ("lds_bytes", C.c_int32), ("full_kernels", C.c_int32),
                ("n_shadow", C.c_int32), ("top_bytes", C.c_int32), ("top_object_nodes", C.c_int32),
                ("top_light_nodes", C.c_int32), ("top_kd_nodes", C.c_int32), ("top_shm", C.c_int32),
                ("accel", C.c_int32), ("wide_nodes", C.c_int32), ("wide_tris", C.c_int32), ("wide_stack", C.c_int32),
                ("wide_depth", C.c_int32), ("top_wide_nodes", C.c_int32)]


STAGE_COUNT = 12  # LUMO_STAGE_COUNT
STAGES = ["camera", "closest", "shade", "shadow", "resolve", "finish", "film", "ring",
          "bd_trace_a", "bd_eval_a", "bd_vis", "bd_paths"]


class Stats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double * STAGE_COUNT), ("launches", C.c_uint64 * STAGE_COUNT),
                ("closest_queries", C.c_uint64), ("shadow_queries", C.c_uint64), ("bounces", C.c_uint64),
                ("aabb_tests", C.c_uint64 * 2), ("kd_nodes", C.c_uint64 * 2), ("tri_tests", C.c_uint64 * 2),
                ("samples_nan", C.c_uint64), ("samples_neg", C.c_uint64), ("samples_large", C.c_uint64),
                ("shadow_resolved", C.c_uint64), ("tail_queries", C.c_uint64),
                ("sorted_bounces", C.c_uint64)]


class ScheduleInfo(C.Structure):
    _fields_ = [("schedule", C.c_int32), ("head_streams", C.c_int32), ("head_bounces", C.c_int32),
                ("merged_passes", C.c_int32), ("units_in_flight", C.c_int32), ("task_groups", C.c_int32),
                ("fused", C.c_int32), ("tail_bounces", C.c_int32)]


SCHED_SEQUENTIAL, SCHED_FUSED_PIPELINE, SCHED_SPLIT_PIPELINE = range(3)
# LUMO_OPT_* (include/lumo_amd.h), by the name Device.set_option takes
OPTIONS = ["timing", "lds_staging", "top_staging", "fused", "tail_below", "pipeline", "heads", "merge_passes",
           "dyn_fetch", "bounce_threads", "split_pipe", "split_groups", "bdpt_tail", "bounce_ahead", "lds_grid",
           "top_grid", "top_kb", "kd_lds", "stack_class", "full_kernels", "poison", "tail_priority", "top_kd",
           "tail_bounces", "film_first", "bdpt_top", "bdpt_groups", "ray_sort", "accel"]
OPT = {name: i for i, name in enumerate(OPTIONS)}


class CameraParams(C.Structure):
    _fields_ = [("origin", C.c_double * 3), ("towards", C.c_double * 3), ("up", C.c_double * 3),
                ("zoom", C.c_double), ("lens_radius", C.c_double), ("focal_length", C.c_double),
                ("vfov", C.c_double), ("width", C.c_int64), ("height", C.c_int64),
                ("illuminant", C.c_int32), ("color_space", C.c_int32),
                ("filter_radius", C.c_double), ("filter_sigma", C.c_double),
                ("camera_type", C.c_int32), ("pad0", C.c_int32)]


class PathDump(C.Structure):
    _fields_ = [("radiance", c_double_p), ("lambda_", c_double_p), ("raster", c_double_p),
                ("depth", c_uint64_p), ("delta", c_double_p)]


# (name, restype, argtypes) of every exported symbol declared in include/*.h
DEVICE_API = [
    ("lumo_create", C.c_int32, [C.c_int, C.POINTER(C.c_void_p)]),
    ("lumo_destroy", None, [C.c_void_p]),
    ("lumo_status_str", C.c_char_p, [C.c_int32]),
    ("lumo_abi_version", C.c_int, []),
    ("lumo_device_count", C.c_int, []),
    ("lumo_scene_upload", C.c_int32, [C.c_void_p, C.POINTER(SceneDesc)]),
    ("lumo_camera_set", C.c_int32, [C.c_void_p, C.POINTER(CameraDesc)]),
    ("lumo_render_tiles", C.c_int32, [C.c_void_p, C.POINTER(TileTask), C.c_size_t, C.POINTER(RenderCfg),
                                      C.POINTER(TileResult)]),
    ("lumo_trace", C.c_int32, [C.c_void_p, C.POINTER(RaySoA), C.c_size_t, C.POINTER(HitSoA), C.c_int]),
    ("lumo_stats_get", C.c_int32, [C.c_void_p, C.POINTER(Stats)]),
    ("lumo_stats_reset", C.c_int32, [C.c_void_p]),
    ("lumo_stats_busy_ms", C.c_int32, [C.c_void_p, C.c_uint32, C.POINTER(C.c_double)]),
    ("lumo_set_option", C.c_int32, [C.c_void_p, C.c_int32, C.c_int64]),
    ("lumo_get_option", C.c_int32, [C.c_void_p, C.c_int32, C.POINTER(C.c_int64)]),
    ("lumo_last_schedule", C.c_int32, [C.c_void_p, C.POINTER(ScheduleInfo)]),
    ("lumo_debug_stream", C.c_int32, [C.c_void_p, C.c_size_t]),
    ("lumo_debug_scan", C.c_int32, [C.c_void_p, c_uint32_p, c_uint32_p, C.c_size_t]),
    ("lumo_scene_info", C.c_int32, [C.c_void_p, C.POINTER(SceneInfo)]),
    ("lumo_debug_set_integrator", C.c_int32, [C.c_void_p, C.c_int]),
    ("lumo_debug_set_sampler", C.c_int32, [C.c_void_p, C.c_int]),
    ("lumo_debug_trace", C.c_int32, [C.c_void_p, C.POINTER(TileTask), C.c_int, C.c_int, c_double_p, C.POINTER(C.c_int)]),
    ("lumo_debug_paths", C.c_int32, [C.c_void_p, C.POINTER(TileTask), C.POINTER(PathDump)]),
]
HOST_API = [
    ("lumo_spectrum_from_rgb", Spectrum, [C.c_double, C.c_double, C.c_double]),
    ("lumo_spectrum_from_srgb", Spectrum, [C.c_int, C.c_int, C.c_int]),
    ("lumo_spectrum_from_pts", Spectrum, [C.c_char_p]),
    ("lumo_rgb2spec_cell", None, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]),
    ("lumo_rgb2spec_write", C.c_int, [C.c_char_p, C.c_int]),
    ("lumo_builder_new", C.c_void_p, []),
    ("lumo_builder_free", None, [C.c_void_p]),
    ("lumo_builder_material_lambertian", C.c_int, [C.c_void_p, Spectrum]),
    ("lumo_builder_material_light", C.c_int, [C.c_void_p, Spectrum, C.c_int, C.c_double, C.c_int]),
    ("lumo_builder_material_microfacet", C.c_int, [C.c_void_p, C.c_double, C.c_double, C.c_double, C.c_int, C.c_int,
                                                   Spectrum, Spectrum, Spectrum]),
    ("lumo_builder_material_diffuse", C.c_int, [C.c_void_p, Spectrum]),
    ("lumo_builder_material_metal", C.c_int, [C.c_void_p, Spectrum, C.c_double, C.c_double, C.c_double]),
    ("lumo_builder_material_transparent", C.c_int, [C.c_void_p, Spectrum, C.c_double, C.c_double]),
    ("lumo_builder_material_mirror", C.c_int, [C.c_void_p]),
    ("lumo_builder_material_glass", C.c_int, [C.c_void_p]),
    ("lumo_builder_empty_box", C.c_int, [C.c_void_p, Spectrum, C.c_int, C.c_int]),
    ("lumo_builder_instance_op", C.c_int, [C.c_void_p, C.c_int, C.c_int64, C.c_int, C.c_double, C.c_double,
                                           C.c_double]),
    ("lumo_builder_count", C.c_int64, [C.c_void_p, C.c_int]),
    ("lumo_builder_add_sphere", C.c_int, [C.c_void_p, C.c_double, C.c_int, C.c_int]),
    ("lumo_builder_set_environment_map", C.c_int, [C.c_void_p, Spectrum, C.c_double]),
    ("lumo_builder_set_environment_texture", C.c_int, [C.c_void_p, C.c_int, C.c_double]),
    ("lumo_builder_texture_solid", C.c_int, [C.c_void_p, Spectrum]),
    ("lumo_builder_texture_image", C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t]),
    ("lumo_builder_texture_hdr", C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t]),
    ("lumo_builder_texture_texels", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(Spectrum), Spectrum]),
    ("lumo_builder_texture_checkerboard", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double]),
    ("lumo_builder_texture_marble", C.c_int, [C.c_void_p, C.c_uint64, Spectrum]),
    ("lumo_builder_texture_mandelbrot", C.c_int, [C.c_void_p]),
    ("lumo_builder_normal_map", C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t]),
    ("lumo_builder_normal_map_texels", C.c_int, [C.c_void_p, C.c_int, C.c_int, c_double_p]),
    ("lumo_builder_material_textured", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    ("lumo_builder_add_file", C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p, C.c_size_t]),
    ("lumo_builder_set_map_ks", C.c_int, [C.c_void_p, C.c_int]),
    ("lumo_builder_add_obj_mesh", C.c_int64, [C.c_void_p, C.c_char_p, C.c_size_t, C.c_int]),
    ("lumo_builder_load_obj_scene", C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]),
    ("lumo_builder_error", C.c_char_p, [C.c_void_p]),
    ("lumo_builder_add_mesh", C.c_int, [C.c_void_p, c_double_p, C.c_int64, c_int64_p, c_int64_p, C.c_int64,
                                        C.c_int, C.c_int]),
    ("lumo_builder_add_rectangle", C.c_int, [C.c_void_p, c_double_p, c_double_p, c_double_p, C.c_int, C.c_int]),
    ("lumo_builder_cornell_box", C.c_void_p, []),
    ("lumo_builder_build", C.c_void_p, [C.c_void_p]),
    ("lumo_scene_get_desc", C.c_int32, [C.c_void_p, C.POINTER(SceneDesc)]),
    ("lumo_scene_free", None, [C.c_void_p]),
    ("lumo_camera_params_default", None, [C.POINTER(CameraParams)]),
    ("lumo_camera_params_cornell_box", None, [C.POINTER(CameraParams)]),
    ("lumo_camera_build", C.c_int32, [C.POINTER(CameraParams), C.POINTER(CameraDesc)]),
    ("lumo_lmath", None, [C.c_int, c_double_p, c_double_p, C.c_int64]),
    ("lumo_make_tasks", C.c_int64, [C.c_int64, C.c_int64, C.c_uint64, C.c_uint64, C.POINTER(TileTask),
                                    C.c_int64]),
]

_lib = None


def load(path=None):
    """Load liblumo_amd.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise OSError(f"lumo_amd: {p} not built; run `make` (or __graft_entry__.build())")
    lib = C.CDLL(p)
    for name, res, args in DEVICE_API + HOST_API:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.lumo_abi_version() != ABI_VERSION:  # a stale build: struct layouts would not match
        raise OSError(f"lumo_amd: {p} has ABI version {lib.lumo_abi_version()}, expected {ABI_VERSION}; rebuild")
    if path is None:
        _lib = lib
    return lib


def check(st, what=""):
    if st != LUMO_OK:
        raise RuntimeError(f"lumo_amd: {what} failed: {STATUS.get(st, st)}")
