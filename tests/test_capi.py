"""CPU tests: libpcops.so loads and exports every symbol include/pcops.h declares
(no compute calls -- there is no GPU here)."""
import ctypes
import os
import re

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "pcops.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pcops_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_binding_table():
    from svdformer_pointsea_amd import _lib

    assert set(_declared()) == set(_lib.exported_symbols())


def test_library_exports_every_declared_symbol():
    from svdformer_pointsea_amd import _lib

    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in _declared():
        assert hasattr(L, name), name
    assert _lib.lib().pcops_abi_version() == 2
    assert _lib.lib().pcops_status_string(0) == b"ok"


def test_library_is_gfx950_code_object():
    from svdformer_pointsea_amd import _lib

    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_size_queries_without_gpu():
    from svdformer_pointsea_amd import _lib

    L = _lib.lib()
    assert L.pcops_fps_workspace_bytes(32, 16384) == 0  # register-resident path
    assert L.pcops_fps_workspace_bytes(2, 20000) == 2 * 20000 * 4
