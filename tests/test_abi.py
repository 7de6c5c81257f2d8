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


def test_library_embeds_the_tree_source_hash():
    """libce_amd.so carries the content hash of the sources it was built from
    (ce_version() "src=..."), equal to the tree's (the Makefile's rule)."""
    from ce_amd import _lib

    lib = _lib.load()
    assert _lib.built_hash(lib.ce_version()) == _lib.source_hash() is not None


def _copy_tree(tmp_path):
    import shutil

    pkg = tmp_path / "consensus-entropy_amd"
    shutil.copytree(os.path.join(PKG_DIR, "ce_amd"), pkg / "ce_amd",
                    ignore=shutil.ignore_patterns("__pycache__"))
    shutil.copytree(os.path.join(PKG_DIR, "csrc"), pkg / "csrc")
    shutil.copytree(os.path.join(ROOT, "include"), tmp_path / "include")
    return pkg


def _load_in(pkg, extra_env=None):
    import sys

    env = {k: v for k, v in os.environ.items() if k != "CE_AMD_LIB"}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, "-c", "import ce_amd; ce_amd.load(); print('loaded')"], cwd=str(pkg),
                          capture_output=True, text=True, timeout=300, env=env)


def test_load_refuses_a_stale_library(tmp_path):
    """One byte flipped in a copied header makes the copied library stale:
    load() refuses it (no silent use of a build of other sources); the
    unmodified copy loads; CE_AMD_LIB naming the library on purpose only
    reports the difference on stderr."""
    pkg = _copy_tree(tmp_path)
    ok = _load_in(pkg)
    assert ok.returncode == 0 and "loaded" in ok.stdout, ok.stderr[-1500:]
    hdr = pkg / "csrc" / "ce_device.hpp"
    b = bytearray(hdr.read_bytes())
    b[100] ^= 0x01
    hdr.write_bytes(bytes(b))
    bad = _load_in(pkg)
    assert bad.returncode != 0 and "stale HIP extension" in bad.stderr, bad.stderr[-1500:]
    swapped = _load_in(pkg, {"CE_AMD_LIB": str(pkg / "ce_amd" / "libce_amd.so")})
    assert swapped.returncode == 0 and "built from other sources" in swapped.stderr, swapped.stderr[-1500:]
