"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU needed)."""
import ctypes as C
import os
import re

import lumo_amd as L
from lumo_amd import _ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    names = set()
    for h in ("lumo_amd.h", "lumo_host.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"\b(lumo_[a-z0-9_]+)\s*\(", txt))
    return names


def test_every_declared_symbol_is_exported():
    lib = C.CDLL(_ffi.LIB_PATH)
    missing = [n for n in sorted(declared()) if not hasattr(lib, n)]
    assert not missing, missing
    assert len(declared()) >= 30


def test_ffi_table_covers_header():
    table = {n for n, _, _ in _ffi.DEVICE_API + _ffi.HOST_API}
    assert declared() <= table, declared() - table


def test_abi_version_and_status_strings():
    lib = L.lib()
    assert lib.lumo_abi_version() == 10 == _ffi.ABI_VERSION
    assert lib.lumo_status_str(0) == b"ok"
    assert lib.lumo_status_str(6) == b"unsupported"


def test_create_without_gpu_fails_loudly():
    lib = L.lib()
    n = lib.lumo_device_count()
    if n > 0:
        return  # covered by the GPU tests
    ctx = C.c_void_p()
    assert lib.lumo_create(0, C.byref(ctx)) == 2  # LUMO_ERR_NO_DEVICE
    assert not ctx.value


def test_null_arguments_rejected():
    lib = L.lib()
    assert lib.lumo_scene_upload(None, None) == 1
    assert lib.lumo_render_tiles(None, None, 0, None, None) == 1
    assert lib.lumo_set_option(None, 0, 1) == 1
    assert lib.lumo_get_option(None, 0, None) == 1
    assert lib.lumo_last_schedule(None, None) == 1


def test_option_table_matches_header():
    """_ffi.OPTIONS lists LUMO_OPT_* in the header's order, and every option has its environment
    variable in the library's table (names only; values need a context, i.e. a GPU)."""
    txt = open(os.path.join(ROOT, "include", "lumo_amd.h")).read()
    body = txt[txt.index("LUMO_OPT_TIMING = 0"):txt.index("LUMO_OPT_COUNT")]
    names = re.findall(r"\bLUMO_OPT_([A-Z_]+)\b", re.sub(r"/\*.*?\*/", "", body, flags=re.S))
    assert [n.lower() for n in names] == _ffi.OPTIONS
    so = open(_ffi.LIB_PATH, "rb").read()
    for env in re.findall(r"\((LUMO_[A-Z_]+), ", body):
        assert env.encode() in so, env
