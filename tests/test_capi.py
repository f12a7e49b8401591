"""CPU-side checks of the C-ABI boundary: the library loads and exports every
function include/*.h declares (no compute calls without a GPU)."""
import glob
import os
import re

from hichap_master_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(hh_\w+)\s*\(", txt, flags=re.M))
    return names


def test_library_loads_and_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    assert declared_functions() == set(_lib.SIGNATURES)


def test_version_and_error_plumbing():
    lib = _lib.load()
    assert lib.hh_version() >= 0x100
    # a NULL-argument call must fail cleanly with a message, not crash
    import ctypes as C
    rc = lib.hh_matrix_get_info(None, None)
    assert rc == -1
    assert b"null" in lib.hh_last_error()


def test_gw_create_refuses_too_many_haplotype_cells():
    # the column sort keeps 32-bit radix offsets: >= 2^32 - 1 cells must be
    # refused before anything touches the device
    import ctypes as C
    import numpy as np
    lib = _lib.load()
    off = np.array([0, 10], dtype=np.int64)
    out = C.c_void_p()
    for fn in (lib.hh_gw_create_device, lib.hh_gw_create):
        rc = fn(None, None, None, 0, C.c_void_p(8), C.c_void_p(8), C.c_void_p(8), (1 << 32) - 1, 10,
                off.ctypes.data_as(C.c_void_p), 1, None, C.byref(out))
        assert rc != 0
        assert b"2^32" in lib.hh_last_error()
        assert not out.value
