"""Helpers shared by the GPU parity tests and smoke()."""
import ctypes as C

import numpy as np

from lumo_amd import _ffi


def gpu_paths(dev, task, sampler=0):
    """lumo_debug_paths: per-path radiance / wavelengths / raster / depth of one task."""
    P = (task.px_max[0] - task.px_min[0]) * (task.px_max[1] - task.px_min[1])
    m = P * task.samples
    rad, lam, ras = np.zeros(4 * m), np.zeros(4 * m), np.zeros(2 * m)
    depth, delta = np.zeros(m, dtype=np.uint64), np.zeros(task.samples)
    dump = _ffi.PathDump(rad.ctypes.data_as(_ffi.c_double_p), lam.ctypes.data_as(_ffi.c_double_p),
                         ras.ctypes.data_as(_ffi.c_double_p), depth.ctypes.data_as(_ffi.c_uint64_p),
                         delta.ctypes.data_as(_ffi.c_double_p))
    lib = _ffi.load()
    _ffi.check(lib.lumo_debug_set_sampler(dev.ctx, int(sampler)), "debug_set_sampler")
    try:
        _ffi.check(lib.lumo_debug_paths(dev.ctx, C.byref(task), C.byref(dump)), "debug_paths")
    finally:
        lib.lumo_debug_set_sampler(dev.ctx, 0)
    return dict(radiance=rad.reshape(-1, 4), lam=lam.reshape(-1, 4), raster=ras.reshape(-1, 2), depth=depth,
                delta=delta)


def oracle_threads():
    """Threads for the CPU oracle in a parity test: the cores this process may use (the affinity
    mask, capped by a cgroup v2 quota: on the GPU box os.cpu_count() is the whole machine)."""
    import math
    import os
    n = len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, math.floor(int(q) / int(period))))
    except (OSError, ValueError):
        pass
    return max(1, min(n, 32))
