"""CPU-side checks of the drop-in boundary: libsli.so builds for gfx950, loads without a GPU, and
exports every entry point include/sli.h declares (no compute calls here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sli_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from simplellminference_amd import build, _lib
    build.build()
    L = ctypes.CDLL(_lib.LIB_PATH)
    names = _declared("sli.h")
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_python_bindings_cover_the_header():
    from simplellminference_amd import _lib
    assert set(_declared("sli.h")) == set(_lib.exported_symbols())


def test_status_strings_without_gpu():
    from simplellminference_amd import _lib
    L = _lib.load()
    assert L.sli_version() == 1
    assert L.sli_status_str(2) == b"shape mismatch"
    assert L.sli_mha_workspace_bytes(2048, 32, 128) > 0
    assert L.sli_comm_id_bytes() == 128
