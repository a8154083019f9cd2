"""C ABI: the HIP library loads on a GPU-less host and exports every symbol
include/burgers.h declares (no compute calls here)."""
import ctypes
import os
import re

from conftest import ROOT


def header_symbols():
    text = open(os.path.join(ROOT, "include", "burgers.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(burg_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from finitedifference_amd import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), f"libburgers_hip.so does not export {s}"
    assert sorted(syms) == sorted(_lib.EXPORTS)


def test_abi_version_and_errors_without_gpu():
    from finitedifference_amd import _lib
    lib = _lib.load()
    assert lib.burg_abi_version() == _lib.ABI_VERSION
    h = ctypes.c_void_p()
    # a null out pointer is rejected before any device call
    assert lib.burg_ctx_create(0, 8, 8, None) == _lib.BURG_EINVAL
    assert b"null" in lib.burg_last_error()
    assert lib.burg_set_options(None, 64, 0, 0.0, 0) == _lib.BURG_EINVAL


def test_built_for_gfx950():
    so = open(os.path.join(ROOT, "finitedifference_amd", "libburgers_hip.so"), "rb").read()
    assert b"gfx950" in so
