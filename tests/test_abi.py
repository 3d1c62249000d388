"""The C ABI library: builds for gfx950, loads, exports every symbol that
include/metacov_amd.h declares, and refuses to run without a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from metacov_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "metacov_amd.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mc_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported(lib_built):
    lib = ctypes.CDLL(lib_built)
    syms = declared_symbols()
    assert len(syms) == len(_lib.SIGNATURES) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    # and the ctypes binding covers exactly the header
    assert set(syms) == set(_lib.SIGNATURES)


def test_gfx950_code_object(lib_built):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", lib_built],
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(lib_built, "rb").read()
    assert b"gfx950" in blob


def test_no_torch_in_abi():
    code = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    assert "torch" not in code.lower() and "at::" not in code and "Tensor" not in code


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="only meaningful without a HIP device")
def test_ctx_create_fails_loudly_without_gpu(lib_built):
    from metacov_amd.engine import CoverageEngine
    with pytest.raises(_lib.MetacovError, match="no HIP device|hip"):
        CoverageEngine(0)


def test_missing_library_is_loud(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.LibraryNotBuilt):
        _lib.load()


def test_library_built_from_this_tree(lib_built):
    """The library's stamped source hash is the tree's (a stale .so would be
    rebuilt by build.build, never silently reused)."""
    from metacov_amd import build
    lib = ctypes.CDLL(lib_built)
    lib.mc_build_id.restype = ctypes.c_char_p
    assert lib.mc_build_id().decode() == "mc-source-sha256:" + build.source_hash()
    assert build.built_hash() == build.source_hash()
