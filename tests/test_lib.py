"""C-ABI library: loads on a CPU-only host and exports every symbol include/bgnn.h declares.
No compute calls (no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bgnn.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bgnn_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("bgnn_graph_build", "bgnn_spmm_fwd", "bgnn_spmm_bwd", "bgnn_sage_fwd", "bgnn_gemm_f32"):
        assert s in syms


def test_library_loads_and_exports_every_declared_symbol():
    from bgnn import _lib

    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.bgnn_abi_version() == _lib.ABI_VERSION
    assert set(declared_symbols()) == set(_lib.SIGNATURES), "ctypes signatures out of sync with the header"


def test_library_is_built_for_gfx950():
    from bgnn import _lib

    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", _lib.LIB_PATH], capture_output=True,
                         text=True)
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob or "gfx950" in out.stdout


def test_csr_struct_layout_matches_header():
    from bgnn import _lib

    assert ctypes.sizeof(_lib.CsrStruct) == 5 * 8 + 2 * 8 + 4 * 4


def test_size_queries_need_no_gpu():
    from bgnn import _lib

    assert _lib.query("bgnn_graph_build_ws_bytes", 1000, 100) > 0
    assert _lib.query("bgnn_sage_fwd_slots", 80656) == 1024
    assert _lib.query("bgnn_gemm_ws_bytes", 80656, 1024, 512, 0, 1) == 0      # forward: no split-K
    assert _lib.query("bgnn_gemm_ws_bytes", 1024, 512, 80656, 1, 0) > 0       # wgrad: split-K


def test_error_string_and_argument_validation():
    from bgnn import _lib

    with pytest.raises(_lib.BgnnError, match="bad transpose"):
        _lib.call("bgnn_gemm_f32", 3, 0, 1, 1, 1, 1.0, None, 1, None, 1, 0.0, None, 1, None, 0, None)
