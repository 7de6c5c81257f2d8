"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
entry point include/ce.h declares (and the Python binding binds exactly those),
host-only functions answer, and the product package never touches the oracle."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import PKG_DIR, ROOT

HEADER = os.path.join(ROOT, "include", "ce.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ce_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from ce_amd import _lib

    lib = _lib.load()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (ce_[a-z_0-9]+)$", out, flags=re.M))
    declared = set(header_functions())
    assert declared, "no declarations parsed"
    assert declared <= exported, sorted(declared - exported)
    assert set(_lib.SIGNATURES) == declared
    for name in declared:
        assert getattr(lib, name) is not None


def test_library_is_gfx950_and_torch_free():
    from ce_amd import _lib

    dyn = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True, text=True).stdout
    # the NEEDED entries only: a hex address in the table may well read "...c10"
    needed = [ln.split("[")[-1].rstrip("]") for ln in dyn.splitlines() if "(NEEDED)" in ln]
    assert needed and not any("torch" in n or n.startswith("libc10") for n in needed), needed
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_host_only_entry_points():
    from ce_amd import _lib

    lib = _lib.load()
    assert lib.ce_version().startswith(b"ce_amd")
    ws = lib.ce_select_mc_workspace_bytes(100_000_000, 10)
    assert 1024 * 10 * 16 <= ws < 1 << 20
    assert lib.ce_select_mix_workspace_bytes(1608, 1300, 10) >= lib.ce_topq_workspace_bytes(1608, 10)
    assert lib.ce_select_batched_workspace_bytes(500 * 1608, 500, 10) >= 500 * 10 * 16


def test_argument_errors_without_gpu():
    """Validation happens before any HIP call, so it is testable here."""
    from ce_amd import _lib

    lib = _lib.load()
    rc = lib.ce_topq(None, 10, -1, 0, None, 0, None, None, None)  # q < 0
    assert rc == _lib.CE_EINVAL and b"q=-1" in lib.ce_last_error()
    rc = lib.ce_select_mc(ctypes.c_void_p(16), 0, 10, 0, 4, 4, 4, 1, 10, 0, None, 0, ctypes.c_void_p(16),
                          ctypes.c_void_p(16), None)  # M = 0
    assert rc == _lib.CE_EINVAL
    rc = lib.ce_select_mc(ctypes.c_void_p(16), 0, 1000, 16, 4, 64, 4, 1, 10, 0, ctypes.c_void_p(256), 8,
                          ctypes.c_void_p(16), ctypes.c_void_p(16), None)  # workspace too small
    assert rc == _lib.CE_EWORKSPACE
    rc = lib.ce_vote_entropy(ctypes.c_void_p(16), 10, 5, 9, 5, None, ctypes.c_void_p(16), None)
    assert rc == _lib.CE_EUNSUPPORTED


def test_product_never_imports_oracle():
    pkg = os.path.join(PKG_DIR, "ce_amd")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert "oracle" not in src.replace("oracle/", ""), f


def test_no_cpu_fallback():
    torch = pytest.importorskip("torch")
    from ce_amd import ops

    with pytest.raises(ValueError, match="HIP device"):
        ops.select_mc(torch.zeros((4, 8, 4)), 2)
