"""ctypes loader for the CPU oracle (test infrastructure only; see oracle/oracle.h)."""
import ctypes as C
import os

import numpy as np

from lumo_amd import _ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "_build", "liblumo_oracle.so")
# the same restatement built against the platform libm instead of lmath.h (sensitivity checks)
ORACLE_GLIBC_PATH = os.path.join(ROOT, "oracle", "_build", "liblumo_oracle_glibc.so")

WAVEFRONT, LUMO_ORDER = 0, 1


class Counters(C.Structure):
    _fields_ = [("aabb_tests", C.c_uint64), ("kd_nodes", C.c_uint64), ("tri_tests", C.c_uint64),
                ("closest_queries", C.c_uint64), ("shadow_queries", C.c_uint64)]


_libs = {}


def load(path=None):
    path = path or ORACLE_PATH
    if path not in _libs:
        lib = C.CDLL(path)
        lib.oracle_render_tiles.restype = C.c_int
        lib.oracle_render_tiles.argtypes = [C.POINTER(_ffi.SceneDesc), C.POINTER(_ffi.CameraDesc),
                                            C.POINTER(_ffi.TileTask), C.c_size_t, C.c_int, C.c_int,
                                            C.POINTER(_ffi.TileResult), C.POINTER(Counters)]
        lib.oracle_trace_paths.restype = C.c_int
        lib.oracle_trace_paths.argtypes = [C.POINTER(_ffi.SceneDesc), C.POINTER(_ffi.CameraDesc),
                                           C.POINTER(_ffi.TileTask), _ffi.c_double_p, _ffi.c_double_p,
                                           _ffi.c_double_p, _ffi.c_uint64_p, _ffi.c_double_p]
        lib.oracle_trace.restype = C.c_int
        lib.oracle_trace.argtypes = [C.POINTER(_ffi.SceneDesc), C.POINTER(_ffi.RaySoA), C.c_size_t,
                                     C.POINTER(_ffi.HitSoA), C.c_int, C.POINTER(Counters)]
        lib.oracle_set_integrator.restype = None
        lib.oracle_set_integrator.argtypes = [C.c_int]
        lib.oracle_set_accel.restype = None
        lib.oracle_set_accel.argtypes = [C.c_int]
        lib.oracle_wide_export.restype = C.c_int
        lib.oracle_wide_export.argtypes = [C.POINTER(_ffi.SceneDesc), C.POINTER(C.c_int64), C.c_void_p,
                                           _ffi.c_double_p, _ffi.c_int32_p, _ffi.c_int32_p]
        lib.oracle_set_sampler.restype = None
        lib.oracle_set_sampler.argtypes = [C.c_int]
        lib.oracle_sampler_points.restype = C.c_int64
        lib.oracle_sampler_points.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, _ffi.c_double_p, C.c_int64]
        lib.oracle_set_tone_map.restype = None
        lib.oracle_set_tone_map.argtypes = [C.c_int, C.c_double]
        dp = _ffi.c_double_p
        lib.oracle_bsdf_sample.restype = C.c_int
        lib.oracle_bsdf_sample.argtypes = [C.POINTER(_ffi.SceneDesc), C.c_int, dp, dp, C.c_size_t, C.c_uint64, dp,
                                           C.POINTER(C.c_int)]
        lib.oracle_bsdf_eval.restype = C.c_int
        lib.oracle_bsdf_eval.argtypes = [C.POINTER(_ffi.SceneDesc), C.c_int, dp, dp, dp, C.c_size_t, dp, dp]
        lib.oracle_furnace.restype = C.c_int
        lib.oracle_furnace.argtypes = [C.POINTER(_ffi.SceneDesc), C.c_int, dp, C.c_size_t, C.c_uint64, dp]
        lib.oracle_light_sample.restype = C.c_int
        lib.oracle_light_sample.argtypes = [C.POINTER(_ffi.SceneDesc), C.c_int, dp, C.c_size_t, C.c_uint64, dp]
        lib.oracle_light_pdf.restype = C.c_int
        lib.oracle_light_pdf.argtypes = [C.POINTER(_ffi.SceneDesc), C.c_int, dp, dp, C.c_size_t, dp]
        lib.oracle_math.restype = C.c_int
        lib.oracle_math.argtypes = [C.c_int, dp, C.c_size_t, dp]
        lib.oracle_mis_sums.restype = C.c_int
        lib.oracle_mis_sums.argtypes = [C.POINTER(_ffi.SceneDesc), C.POINTER(_ffi.CameraDesc), C.c_size_t, C.c_uint64,
                                        dp, _ffi.c_int32_p]
        _libs[path] = lib
    return _libs[path]


def render_tasks(scene_desc, camera_desc, tasks, mode=WAVEFRONT, threads=1, path=None, tone_map=(0, 0.0),
                 integrator=0, splats_out=None, sampler=0, accel=0):
    """Returns (list of rgb_w arrays, results array, counters).  With integrator = 1 (BDPT) the
    per-task light-tracing splats are appended to `splats_out` (a list) as (x, y, rgb) arrays.
    sampler: lumo_amd.SamplerType (samplers.rs:6-17).  accel: 0 lumo's structures, 1 the wide BVH
    (LUMO_OPT_ACCEL)."""
    lib = load(path)
    lib.oracle_set_accel(int(accel))
    try:
        return _render_tasks(lib, scene_desc, camera_desc, tasks, mode, threads, tone_map, integrator, splats_out,
                             sampler)
    finally:
        lib.oracle_set_accel(0)


def _render_tasks(lib, scene_desc, camera_desc, tasks, mode, threads, tone_map, integrator, splats_out, sampler):
    lib.oracle_set_tone_map(*tone_map)
    lib.oracle_set_integrator(integrator)
    lib.oracle_set_sampler(int(sampler))
    n = len(tasks)
    arr = tasks if isinstance(tasks, C.Array) else (_ffi.TileTask * n)(*tasks)
    caps = [16 * (t.px_max[0] - t.px_min[0]) * (t.px_max[1] - t.px_min[1]) * t.samples if integrator else 0
            for t in arr]
    while True:
        res = (_ffi.TileResult * n)()
        bufs, sbufs = [], []
        for i, t in enumerate(arr):
            P = (t.px_max[0] - t.px_min[0]) * (t.px_max[1] - t.px_min[1])
            b = np.zeros(4 * P)
            bufs.append(b)
            res[i].rgb_w = b.ctypes.data_as(_ffi.c_double_p)
            sb = (_ffi.Splat * max(caps[i], 1))()
            sbufs.append(sb)
            res[i].splats = sb
            res[i].splat_cap = caps[i]
        cnt = Counters()
        st = lib.oracle_render_tiles(C.byref(scene_desc), C.byref(camera_desc), arr, n, mode, threads, res,
                                     C.byref(cnt))
        if st == 7:  # LUMO_ERR_OOM: splat buffers too small, retry with the reported counts
            caps = [max(c, r.num_splats) for c, r in zip(caps, res)]
            continue
        if st != 0:
            lib.oracle_set_integrator(0)
            lib.oracle_set_sampler(0)
        assert st == 0, st
        break
    lib.oracle_set_integrator(0)
    lib.oracle_set_sampler(0)
    if splats_out is not None:
        for i in range(n):
            m = res[i].num_splats
            a = np.ctypeslib.as_array(sbufs[i])[:m] if m else np.zeros(0, dtype=[("x", "<u4"), ("y", "<u4"),
                                                                               ("rgb", "<f8", (3,))])
            splats_out.append(a.copy())
    return bufs, res, cnt


def trace_paths(scene_desc, camera_desc, task, path=None, integrator=0, sampler=0, accel=0):
    lib = load(path)
    lib.oracle_set_integrator(integrator)
    lib.oracle_set_sampler(int(sampler))
    lib.oracle_set_accel(int(accel))
    P = (task.px_max[0] - task.px_min[0]) * (task.px_max[1] - task.px_min[1])
    m = P * task.samples
    rad, lam, ras = np.zeros(4 * m), np.zeros(4 * m), np.zeros(2 * m)
    depth, delta = np.zeros(m, dtype=np.uint64), np.zeros(task.samples)
    st = lib.oracle_trace_paths(C.byref(scene_desc), C.byref(camera_desc), C.byref(task),
                                rad.ctypes.data_as(_ffi.c_double_p), lam.ctypes.data_as(_ffi.c_double_p),
                                ras.ctypes.data_as(_ffi.c_double_p), depth.ctypes.data_as(_ffi.c_uint64_p),
                                delta.ctypes.data_as(_ffi.c_double_p))
    lib.oracle_set_integrator(0)
    lib.oracle_set_sampler(0)
    lib.oracle_set_accel(0)
    assert st == 0, st
    return dict(radiance=rad.reshape(-1, 4), lam=lam.reshape(-1, 4), raster=ras.reshape(-1, 2), depth=depth,
                delta=delta)


def trace(scene_desc, origins, dirs, lights=None, accel=0, with_prim=False):
    """Scene::hit (lights None) or Scene::hit_light per ray: (t, kind, object, counters), with the
    triangle (wide accel only; -1 otherwise) before the counters when with_prim."""
    lib = load()
    n = len(origins)
    o = np.ascontiguousarray(origins, dtype=np.float64)
    d = np.ascontiguousarray(dirs, dtype=np.float64)
    li = np.ascontiguousarray(lights if lights is not None else np.zeros(n), dtype=np.int32)
    rays = _ffi.RaySoA(o.ctypes.data_as(_ffi.c_double_p), d.ctypes.data_as(_ffi.c_double_p), None,
                       li.ctypes.data_as(_ffi.c_int32_p))
    t = np.zeros(n)
    kind, obj, prim = (np.zeros(n, dtype=np.int32) for _ in range(3))
    hits = _ffi.HitSoA(t.ctypes.data_as(_ffi.c_double_p), kind.ctypes.data_as(_ffi.c_int32_p),
                       obj.ctypes.data_as(_ffi.c_int32_p), prim.ctypes.data_as(_ffi.c_int32_p))
    cnt = Counters()
    lib.oracle_set_accel(int(accel))
    try:
        st = lib.oracle_trace(C.byref(scene_desc), C.byref(rays), n, C.byref(hits), int(lights is not None),
                              C.byref(cnt))
    finally:
        lib.oracle_set_accel(0)
    assert st == 0
    if with_prim:
        return t, kind, obj, prim, cnt
    return t, kind, obj, cnt


def _dp(a):
    return a.ctypes.data_as(_ffi.c_double_p)


def bsdf_sample(scene_desc, material, wo, lam, n, seed):
    wo = np.ascontiguousarray(wo, dtype=np.float64)
    lam = np.ascontiguousarray(lam, dtype=np.float64)
    wi = np.zeros((n, 3))
    ok = np.zeros(n, dtype=np.int32)
    st = load().oracle_bsdf_sample(C.byref(scene_desc), material, _dp(wo), _dp(lam), n, seed, _dp(wi),
                                   ok.ctypes.data_as(C.POINTER(C.c_int)))
    assert st == 0
    return wi, ok.astype(bool)


def bsdf_eval(scene_desc, material, wo, lam, wi):
    wo = np.ascontiguousarray(wo, dtype=np.float64)
    lam = np.ascontiguousarray(lam, dtype=np.float64)
    wi = np.ascontiguousarray(wi, dtype=np.float64).reshape(-1, 3)
    pdf = np.zeros(len(wi))
    f = np.zeros((len(wi), 4))
    st = load().oracle_bsdf_eval(C.byref(scene_desc), material, _dp(wo), _dp(lam), _dp(wi), len(wi), _dp(pdf), _dp(f))
    assert st == 0
    return pdf, f


def furnace(scene_desc, material, wo, n, seed):
    wo = np.ascontiguousarray(wo, dtype=np.float64)
    out = np.zeros(4)
    assert load().oracle_furnace(C.byref(scene_desc), material, _dp(wo), n, seed, _dp(out)) == 0
    return out


def light_sample(scene_desc, light, xo, n, seed):
    xo = np.ascontiguousarray(xo, dtype=np.float64)
    wi = np.zeros((n, 3))
    assert load().oracle_light_sample(C.byref(scene_desc), light, _dp(xo), n, seed, _dp(wi)) == 0
    return wi


def light_pdf(scene_desc, light, xo, wi):
    xo = np.ascontiguousarray(xo, dtype=np.float64)
    wi = np.ascontiguousarray(wi, dtype=np.float64).reshape(-1, 3)
    pdf = np.zeros(len(wi))
    assert load().oracle_light_pdf(C.byref(scene_desc), light, _dp(xo), _dp(wi), len(wi), _dp(pdf)) == 0
    return pdf


def mis_sums(scene_desc, camera_desc, n, seed):
    """Per path: the sum of mis::weight over its strategies (mis_tests.rs test_scene) and its length."""
    lib = load()
    sums = np.zeros(n)
    lens = np.zeros(n, dtype=np.int32)
    st = lib.oracle_mis_sums(C.byref(scene_desc), C.byref(camera_desc), n, seed, _dp(sums),
                             lens.ctypes.data_as(_ffi.c_int32_p))
    assert st == 0, st
    return sums, lens


MATH_IO = {0: (3, 6), 1: (6, 3), 2: (4, 10), 3: (3, 4), 4: (6, 1)}


def math(op, x):
    """oracle_math probe `op` over the rows of x (see oracle.cpp)."""
    ni, no = MATH_IO[op]
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1, ni)
    out = np.zeros((len(x), no))
    assert load().oracle_math(op, _dp(x), len(x), _dp(out)) == 0
    return out


def sampler_points(sampler, batch, samples, seed):
    """SamplerType::new(batch, samples, seed) of the oracle, all its points as an (n, 2) array."""
    lib = load()
    lib.oracle_set_sampler(int(sampler))
    out = np.zeros(2 * 256)
    n = lib.oracle_sampler_points(batch, samples, seed, out.ctypes.data_as(_ffi.c_double_p), 256)
    lib.oracle_set_sampler(0)
    assert n >= 0, n
    return out[:2 * n].reshape(-1, 2)


# wide BVH node (lumo_amd/csrc/common/wbvh.h Node, 128 B)
WNODE = np.dtype([("lo", "<f4", (3, 4)), ("hi", "<f4", (3, 4)), ("ref", "<i4", 4), ("n", "<i4"), ("pad", "<i4", 3)])


def wide_export(scene_desc):
    """The wide BVH the upload builds for the scene: dict with ok, nodes (WNODE array), tv
    (records x 10 doubles; column 9 holds (tri, obj) int32 pairs), tri / obj ids, the roots and the
    per object / light BLAS roots, stack need and depth."""
    lib = load()
    info = (C.c_int64 * 8)()
    assert lib.oracle_wide_export(C.byref(scene_desc), info, None, None, None, None) == 0
    nn, nt = int(info[1]), int(info[2])
    nodes = np.zeros(max(nn, 1), dtype=WNODE)
    tv = np.zeros((max(nt, 1), 10))
    ob = np.zeros(max(scene_desc.num_objects, 1), dtype=np.int32)
    lb = np.zeros(max(scene_desc.num_lights, 1), dtype=np.int32)
    assert lib.oracle_wide_export(C.byref(scene_desc), info, nodes.ctypes.data_as(C.c_void_p), _dp(tv),
                                  ob.ctypes.data_as(_ffi.c_int32_p), lb.ctypes.data_as(_ffi.c_int32_p)) == 0
    ids = tv[:, 9].copy().view(np.int32).reshape(-1, 2)
    return dict(ok=bool(info[0]), nodes=nodes[:nn], tv=tv[:nt], tri=ids[:nt, 0], obj=ids[:nt, 1],
                stack=int(info[3]), depth=int(info[4]), obj_root=int(info[5]), light_root=int(info[6]),
                obj_blas=ob[:scene_desc.num_objects], light_blas=lb[:scene_desc.num_lights])
