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
    # light-row blocks of the kernel that will run + one slot per heavy row
    def csr(n_rows, nnz, n_heavy, n_chunks, group_rows=0, n_groups=0, grow=None):
        plan = 1 if group_rows else None
        return _lib.CsrStruct(rowptr=1, col=1, heavy_row=1, heavy_chunk0=1, chunk_heavy=1, n_rows=n_rows, nnz=nnz,
                              n_heavy=n_heavy, n_chunks=n_chunks, chunk=64, gsrc=plan, gmask=plan, gcnt=plan,
                              grow=grow, n_groups=n_groups, group_rows=group_rows)

    q = lambda c: _lib.query("bgnn_sage_fwd_slots", ctypes.byref(c))   # noqa: E731
    assert q(csr(80656, 715872, 0, 0)) == 1024                       # sweep kernel: 1024 blocks
    assert q(csr(80672, 792992, 16, 1264, group_rows=4)) == 1024 + 16   # row-group kernel + heavy rows
    assert q(csr(1000, 8000, 0, 0, group_rows=4)) == 64              # 250 groups, one per wave
    assert q(csr(1000, 8000, 0, 0, group_rows=4, n_groups=40, grow=1)) == 16   # explicit group starts
    # f16x3 (default): a 256-B head for the operand maxima, plus split-K slabs where used
    assert _lib.query("bgnn_gemm_ws_bytes", 80656, 1024, 512, 0, 1) == 256    # forward: no split-K
    assert _lib.query("bgnn_gemm_ws_bytes", 1024, 512, 80656, 1, 0) > 256     # wgrad: split-K
    _lib.call("bgnn_set_tuning", 5, 0)
    try:
        assert _lib.query("bgnn_gemm_ws_bytes", 80656, 1024, 512, 0, 1) == 0  # f32 MFMA: no head
    finally:
        _lib.call("bgnn_set_tuning", 5, 2)


def test_error_string_and_argument_validation():
    from bgnn import _lib

    with pytest.raises(_lib.BgnnError, match="bad transpose"):
        _lib.call("bgnn_gemm_f32", 3, 0, 1, 1, 1, 1.0, None, 1, None, 1, 0.0, None, 1, None, 0, None)
