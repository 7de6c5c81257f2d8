"""ctypes binding of the C-ABI in include/ce.h (libce_amd.so, built for gfx950).

torch is imported first on purpose: torch ships its own libamdhip64.so.7, and
loading libce_amd.so after it makes the dynamic loader reuse that runtime
(same SONAME) instead of mapping a second HIP runtime into the process, so
torch's streams and allocations are valid handles for the engine.
"""
from __future__ import annotations

import ctypes
import os
import threading

try:  # noqa: SIM105 -- see module docstring
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is part of this image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
# CE_AMD_LIB: an alternative build of the same ABI (A/B runs of kernel variants)
LIB_PATH = os.environ.get("CE_AMD_LIB") or os.path.join(_HERE, "libce_amd.so")

CE_OK, CE_EINVAL, CE_EWORKSPACE, CE_ELAUNCH, CE_EUNSUPPORTED = 0, -1, -2, -3, -4
CE_F32, CE_F64, CE_BF16 = 0, 1, 2
CE_MAX_Q = 2048  # the list kernels' q; any larger q runs on the sort path (include/ce.h)

# name -> (restype, argtypes); the exact export list of include/ce.h
_vp, _i64, _i32, _sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_size_t
_int, _cstr = ctypes.c_int, ctypes.c_char_p
SIGNATURES = {
    "ce_last_error": (_cstr, []),
    "ce_version": (_cstr, []),
    "ce_last_kernel": (_cstr, []),
    "ce_committee_entropy": (_int, [_vp, _int, _i64, _i32, _i32, _i64, _i64, _i64, _vp, _vp, _vp]),
    "ce_vote_entropy": (_int, [_vp, _i64, _i32, _i32, _i64, _vp, _vp, _vp]),
    "ce_va_entropy": (_int, [_vp, _i64, _i32, _vp, _vp, _vp]),
    "ce_gnb_predict_proba": (_int, [_vp, _i64, _i32, _i64, _vp, _vp, _vp, _i32, _vp, _i64, _vp]),
    "ce_sgd_predict_proba": (_int, [_vp, _i64, _i32, _i64, _vp, _vp, _i32, _i32, _vp, _i64, _vp]),
    "ce_xgb_predict_proba": (_int, [_vp, _int, _i64, _i32, _i64, _vp, _vp, _vp, _i32, _i32, ctypes.c_float, _i32,
                                    _vp, _int, _i64, _vp]),
    "ce_xgb_lane_table": (_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp]),
    "ce_xgb_predict_proba_lanes": (_int, [_vp, _int, _i64, _i32, _i64, _vp, _i32, _vp, _i32, _i32, ctypes.c_float, _i32,
                                          _vp, _int, _i64, _vp]),
    "ce_xgb_lds_bytes": (_sz, [_i32, _i32]),
    "ce_xgb_expf": (_int, [_vp, _i64, _vp, _vp]),
    "ce_log_f64": (_int, [_vp, _i64, _vp, _vp]),
    "ce_log_f64_host": (_int, [_vp, _i64, _vp]),
    "ce_exp_f64": (_int, [_vp, _i64, _vp, _vp]),
    "ce_exp_f64_host": (_int, [_vp, _i64, _vp]),
    "ce_approx_entropy": (_int, [_vp, _i64, _i32, _vp, _vp, _vp]),
    "ce_wide_approx_entropy": (_int, [_vp, _i64, _i32, _int, _vp, _vp, _vp]),
    "ce_row_div_f64": (_int, [_vp, _vp, _i64, _vp, _vp]),
    "ce_segment_mean": (_int, [_vp, _int, _i64, _i32, _i64, _vp, _vp, _i64, _vp, _int, _i64, _vp]),
    "ce_select_frames_workspace_bytes": (_sz, [_i64, _i32]),
    "ce_select_frames": (_int, [_vp, _i32, _i32, _vp, _vp, _i64, _i32, _i64, _vp, _sz, _vp, _vp, _vp]),
    "ce_topq_workspace_bytes": (_sz, [_i64, _i32]),
    "ce_topq": (_int, [_vp, _i64, _i32, _i64, _vp, _sz, _vp, _vp, _vp]),
    "ce_topq_merge": (_int, [_vp, _vp, _i32, _i32, _vp, _vp, _vp]),
    "ce_select_mc_workspace_bytes": (_sz, [_i64, _i32]),
    "ce_select_mc": (_int, [_vp, _int, _i64, _i32, _i32, _i64, _i64, _i64, _i32, _i64, _vp, _sz, _vp, _vp, _vp]),
    "ce_select_mc_partial": (_int, [_vp, _int, _i64, _i32, _i32, _i64, _i64, _i64, _i32, _i64, _vp, _sz, _vp]),
    "ce_select_finish": (_int, [_i64, _i32, _vp, _sz, _vp, _vp, _vp]),
    "ce_select_finish_cands": (_int, [_i64, _i32, _vp, _sz, _vp, _vp]),
    "ce_merge_cands": (_int, [_vp, _i32, _i32, _vp, _vp, _vp]),
    "ce_select_mc_cands": (_int, [_vp, _int, _i64, _i32, _i32, _i64, _i64, _i64, _i32, _i64, _vp, _sz, _vp, _vp]),
    "ce_select_mc_chunk_workspace_bytes": (_sz, [_i64, _i32]),
    "ce_select_mc_chunk": (_int, [_vp, _int, _i64, _i32, _i32, _i64, _i64, _i64, _i32, _i64, _vp, _i32, _vp, _sz,
                                  _vp]),
    "ce_excl_words": (_sz, [_i64]),
    "ce_select_mc_excl": (_int, [_vp, _int, _i64, _i32, _i32, _i64, _i64, _i64, _vp, _i32, _i64, _vp, _sz, _vp, _vp,
                                 _vp]),
    "ce_mark_selected": (_int, [_vp, _i64, _vp, _i32, _i64, _vp]),
    "ce_select_mix_workspace_bytes": (_sz, [_i64, _i64, _i32]),
    "ce_select_mix": (_int, [_vp, _int, _i64, _i32, _i32, _i64, _i64, _i64, _vp, _i64, _i64, _i32, _vp, _sz,
                             _vp, _vp, _vp]),
    "ce_select_batched_workspace_bytes": (_sz, [_i64, _i32, _i32]),
    "ce_select_batched": (_int, [_vp, _int, _i64, _i32, _i32, _i64, _i64, _i64, _vp, _i32, _i32, _vp, _sz, _vp,
                                 _vp, _vp]),
}

_lib = None
_lock = threading.Lock()


class CEError(RuntimeError):
    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


def source_hash(pkg_dir=_PKG):
    """The content hash of the engine's sources in this tree, by the Makefile's
    rule (SRC_HASH): sha256 over the sorted csrc/*.hip, csrc/*.hpp files, then
    include/ce.h, concatenated; the first 16 hex digits.  None when the tree
    holds no sources (an installed copy)."""
    import hashlib

    csrc = os.path.join(pkg_dir, "csrc")
    header = os.path.join(os.path.dirname(pkg_dir), "include", "ce.h")
    if not os.path.isdir(csrc) or not os.path.isfile(header):
        return None
    h = hashlib.sha256()
    for f in sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".hpp"))) + [None]:
        with open(header if f is None else os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def built_hash(version):
    """The source hash a library embeds in ce_version() ("... src=<hash>"), or None."""
    v = version.decode(errors="replace") if isinstance(version, bytes) else str(version)
    return v.split("src=", 1)[1].split()[0] if "src=" in v else None


def verify_source(lib, path, pkg_dir=_PKG, explicit=False):
    """Refuse a library built from other sources than the tree's (a stale or
    swapped build).  explicit (CE_AMD_LIB named the library on purpose): report
    the difference on stderr instead."""
    tree = source_hash(pkg_dir)
    if tree is None:
        return
    got = built_hash(lib.ce_version())
    if got == tree:
        return
    msg = (f"{path} was built from other sources (its ce_version() says src={got}, the tree's "
           f"{os.path.join(pkg_dir, 'csrc')} + include/ce.h hash to {tree})")
    if explicit:
        import sys

        print(f"ce_amd: note: CE_AMD_LIB: {msg}", file=sys.stderr)
        return
    raise RuntimeError(f"stale HIP extension: {msg}; rebuild it (`make -C consensus-entropy_amd`). "
                       "There is no CPU fallback.")


def load():
    """Load libce_amd.so.  Raises (never falls back) when it is missing or was
    built from other sources than the tree's (ce_version() hash, verify_source)."""
    global _lib
    with _lock:
        if _lib is None:
            explicit = bool(os.environ.get("CE_AMD_LIB"))
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"HIP extension not built: {LIB_PATH} is missing "
                    "(run `python -c 'import __graft_entry__ as g; g.build()'` or "
                    "`make -C consensus-entropy_amd`). There is no CPU fallback.")
            lib = ctypes.CDLL(LIB_PATH)
            missing = []
            for name, (res, args) in SIGNATURES.items():
                try:
                    f = getattr(lib, name)
                except AttributeError:
                    if explicit:  # an older A/B build: bind what it exports, and say what it lacks
                        missing.append(name)
                        continue
                    raise
                f.restype = res
                f.argtypes = args
            if missing:
                import sys

                print(f"ce_amd: note: CE_AMD_LIB={LIB_PATH} lacks {', '.join(missing)}", file=sys.stderr)
            verify_source(lib, LIB_PATH, explicit=explicit)
            _lib = lib
    return _lib


_capture_info = None


def hip_stream_capture_info(stream, status, capture_id):
    """hipStreamGetCaptureInfo(stream, &status, &id) of the HIP runtime the
    engine links (the one torch loaded): 0 = success.  The graph-workspace
    cache keys a capture's workspace by this id (ops._WorkspaceCache)."""
    global _capture_info
    if _capture_info is None:
        f = load().hipStreamGetCaptureInfo  # resolved through libce_amd.so's own dependency
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_ulonglong)]
        _capture_info = f
    return _capture_info(ctypes.c_void_p(stream), ctypes.byref(status), ctypes.byref(capture_id))


def call(name, *args):
    """Call a CE_* returning entry point; raise on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != CE_OK:
        msg = lib.ce_last_error().decode(errors="replace")
        if rc == CE_EINVAL:
            raise ValueError(f"{name}: {msg}")
        raise CEError(name, rc, msg)
    return rc
