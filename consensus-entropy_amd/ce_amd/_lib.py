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


def load():
    """Load libce_amd.so.  Raises (never falls back) when it is missing."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"HIP extension not built: {LIB_PATH} is missing "
                    "(run `python -c 'import __graft_entry__ as g; g.build()'` or "
                    "`make -C consensus-entropy_amd`). There is no CPU fallback.")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                try:
                    f = getattr(lib, name)
                except AttributeError:
                    if os.environ.get("CE_AMD_LIB"):  # an older A/B build: bind what it exports
                        continue
                    raise
                f.restype = res
                f.argtypes = args
            _lib = lib
    return _lib


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
