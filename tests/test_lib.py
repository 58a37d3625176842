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


def test_csr_struct_layout_matches_header(tmp_path):
    """The ctypes mirror of bgnn_csr_t has the C compiler's size and field offsets."""
    import shutil
    import subprocess

    from bgnn import _lib

    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    names = [f[0] for f in _lib.CsrStruct._fields_]
    src = tmp_path / "layout.c"
    src.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"bgnn.h\"\nint main(void){\n"
                   + 'printf("%zu\\n", sizeof(bgnn_csr_t));\n'
                   + "".join(f'printf("%zu\\n", offsetof(bgnn_csr_t, {n}));\n' for n in names) + "return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(_lib.CsrStruct)
    for n, off in zip(names, vals[1:]):
        assert getattr(_lib.CsrStruct, n).offset == off, n


def test_size_queries_need_no_gpu():
    from bgnn import _lib

    assert _lib.query("bgnn_graph_build_ws_bytes", 1000, 100) > 0
    assert _lib.query("bgnn_sage_fwd_slots", 80656) == 1024
    # f16x3 (default): a 256-B head for the operand maxima, plus split-K slabs where used
    assert _lib.query("bgnn_gemm_ws_bytes", 80656, 1024, 512, 0, 1) == 256    # forward: no split-K
    assert _lib.query("bgnn_gemm_ws_bytes", 1024, 512, 80656, 1, 0) > 256     # wgrad: split-K
    _lib.call("bgnn_set_tuning", 5, 1)
    try:
        assert _lib.query("bgnn_gemm_ws_bytes", 80656, 1024, 512, 0, 1) == 0  # bf16x6: no head
    finally:
        _lib.call("bgnn_set_tuning", 5, 2)


def test_error_string_and_argument_validation():
    from bgnn import _lib

    with pytest.raises(_lib.BgnnError, match="bad transpose"):
        _lib.call("bgnn_gemm_f32", 3, 0, 1, 1, 1, 1.0, None, 1, None, 1, 0.0, None, 1, None, 0, None)
