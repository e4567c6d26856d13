"""CPU-only checks of the C ABI boundary: the library loads and exports exactly
what include/grf.h declares (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "grf.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(grf_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    from grf_amd import _lib
    assert declared_functions() == _lib.exported_symbols()


def test_library_exports_every_symbol():
    from grf_amd import _lib
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.grf_version() == _lib.ABI_VERSION
    # host-only helpers are callable without a GPU
    assert [lib.grf_chunk_bounds(10, 3, c) for c in range(3)] == [0, 4, 7]
    assert lib.grf_scan_workspace_bytes(100) == 0
    assert lib.grf_scan_workspace_bytes(10_000_000) > 0
    assert lib.grf_device_count() == 0 or lib.grf_device_count() >= 1


def test_kernels_are_gfx950_code_objects():
    from grf_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_loader_refuses_another_abi_revision(monkeypatch):
    """_lib.load() checks grf_version() against the binding's ABI_VERSION before binding any symbol: a
    library built from other sources (argument lists shift between revisions) raises ImportError."""
    from grf_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "ABI_VERSION", _lib.ABI_VERSION + 1)
    import pytest
    with pytest.raises(ImportError, match="ABI revision"):
        _lib.load()
