"""Device-tensor operators over the C-ABI (torch is plumbing: memory + streams).

Every op takes torch tensors resident on a HIP device, launches on torch's
current stream and returns device tensors; nothing is synchronised here.
There is no CPU path: a CPU tensor is an error.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch

from . import _lib
from ._lib import CE_BF16, CE_F32, CE_F64, call

_DT = {torch.float32: CE_F32, torch.float64: CE_F64, torch.bfloat16: CE_BF16}
LAYOUTS = ("MNC", "NMC")


def _stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _on_gpu(t, what):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{what} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{what} must live on a HIP device (got {t.device}); there is no CPU path")


WS_HEADER_BYTES = 65536 + 256  # include/ce.h: the 64 KiB counter header (+ the 256-B alignment carve)


def new_workspace(nbytes, device, header_only=False):
    """A workspace for the engine, zero-filled as include/ce.h requires (its
    header holds the tiled kernels' arrival counters, which every call leaves
    zero again).  header_only: zero just the header -- for the sort path's
    per-call workspaces, whose body every pass writes before it reads."""
    n = max(int(nbytes), 256)
    if not header_only:
        return torch.zeros(n, dtype=torch.uint8, device=device)
    buf = torch.empty(n, dtype=torch.uint8, device=device)
    buf[:WS_HEADER_BYTES].zero_()
    return buf


class _GraphArena:
    """Zero-filled device memory that captured selections carve their
    workspaces from, one arena per device, filled and synchronised ONCE,
    eagerly, outside any capture.

    A captured call's workspace header (the arrival counters) must be zero at
    the graph's first replay; every call leaves it zero again (include/ce.h).
    Carving from memory zeroed before the capture therefore needs no zero-fill
    node in the graph: each replay runs the selection kernel alone.  A carve is
    never handed out twice, and it is never freed, because a graph may replay
    for the life of the process.  Captures are rare (one per graph) and a small
    pool's workspace is 70-230 KB, so the default 64 MiB lasts hundreds of
    captures.  reserve() adds room before a capture that needs more."""

    ALIGN = 256
    DEFAULT_BYTES = int(os.environ.get("CE_AMD_GRAPH_ARENA_MB", "64")) << 20

    def __init__(self):
        self._free = {}  # device index -> list of [buffer, next offset]

    def reserve(self, device, nbytes):
        """Eager only: make sure `nbytes` can be carved on `device` (adds a
        new zeroed arena when the current ones are short)."""
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("reserve_graph_workspace must run outside HIP-graph capture")
        arenas = self._free.setdefault(device.index, [])
        if any(buf.numel() - off >= nbytes for buf, off in arenas):
            return
        n = max(int(nbytes) + self.ALIGN, self.DEFAULT_BYTES)
        buf = torch.zeros(n, dtype=torch.uint8, device=device)
        # the one synchronisation: the fill must be done before any replay,
        # and a replay may run on any stream
        torch.cuda.current_stream(device).synchronize()
        arenas.append([buf, 0])

    def ensure(self, device):
        if device.index not in self._free:
            self.reserve(device, 0)

    def carve(self, device, nbytes):
        """A zero-filled region of >= nbytes that nothing else uses, or None."""
        nbytes = max(int(nbytes), 256)
        for slot in self._free.get(device.index, ()):
            buf, off = slot
            if buf.numel() - off >= nbytes:
                slot[1] = off + (nbytes + self.ALIGN - 1) // self.ALIGN * self.ALIGN
                return buf[off:off + nbytes]
        return None


def _capture_id(device):
    """The HIP capture id of the device's current stream (unique per capture)."""
    st = ctypes.c_int(0)
    cid = ctypes.c_ulonglong(0)
    rc = _lib.hip_stream_capture_info(torch.cuda.current_stream(device).cuda_stream, st, cid)
    return cid.value if rc == 0 else None


class _WorkspaceCache:
    """Scratch reused across calls, one per (device, stream): include/ce.h
    allows one workspace per stream -- its header holds the arrival counters of
    the folded merges, so two streams sharing one would mix their tickets.  A
    buffer grows (never shrinks), so steady state allocates nothing.

    Bounded: at most MAX_STREAMS buffers, least recently used evicted first (a
    caller cycling through short-lived streams does not pin one buffer per
    stream; an evicted buffer goes back to torch's allocator in its own
    stream's order).  Workspaces of the sort path (q > CE_MAX_Q, ~40 B per
    item: GBs on a 100M pool) are never cached: each such call gets its own,
    released when the call's tensors are, so one large-q call does not keep
    them allocated for the life of the process.

    Under HIP-graph capture a call never uses a cached buffer, so growing the
    cache later cannot free memory a graph still uses, and replays never share
    counters with eager calls.  The workspace is carved from the pre-zeroed
    graph arena (_GraphArena): one carve per (capture, stream), shared by the
    sequential calls on that stream inside that capture, as eager calls share
    their stream's buffer.  The replays then run no zero-fill node.  When the
    arena has no room (or no eager call ever created it), the call falls back
    to a workspace allocated inside the capture with a captured zero fill that
    runs at every replay (correct, one node slower; warned once).  Sort-path
    calls under capture always take that fallback with a header-only fill."""

    MAX_STREAMS = 16

    def __init__(self):
        import collections

        self._ws = collections.OrderedDict()
        self._captured = {}  # (device, stream, capture id) -> carved workspace
        self.arena = _GraphArena()
        self._warned = False

    def get(self, device, nbytes, transient=False):
        device = torch.device(device)
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        with torch.cuda.device(device):  # the capture state of THIS device's current stream
            capturing = torch.cuda.is_current_stream_capturing()
        if capturing:
            return self._get_captured(device, nbytes, transient)
        if transient:
            return new_workspace(nbytes, device, header_only=True)
        self.arena.ensure(device)
        key = (device.index, torch.cuda.current_stream(device).cuda_stream)
        buf = self._ws.get(key)
        if buf is None or buf.numel() < nbytes:
            # the old buffer (if any) is released on this stream: the caching
            # allocator reuses its block only in this stream's order
            buf = new_workspace(nbytes, device)
            self._ws[key] = buf
        self._ws.move_to_end(key)
        while len(self._ws) > self.MAX_STREAMS:
            self._ws.popitem(last=False)
        return buf

    def _get_captured(self, device, nbytes, transient):
        if not transient:
            cid = _capture_id(device)
            key = (device.index, torch.cuda.current_stream(device).cuda_stream, cid)
            buf = self._captured.get(key) if cid is not None else None
            if buf is not None and buf.numel() >= nbytes:
                return buf
            buf = self.arena.carve(device, nbytes) if cid is not None else None
            if buf is not None:
                self._captured[key] = buf
                return buf
            if not self._warned:
                import warnings

                warnings.warn("ce_amd: no pre-zeroed graph workspace left (call ops.reserve_graph_workspace "
                              "before capture); this captured selection replays a zero-fill node", stacklevel=3)
                self._warned = True
        return new_workspace(nbytes, device, header_only=transient)

    def clear(self):
        """Release the cached eager workspaces (the graph arena stays: graphs
        may still replay from it)."""
        self._ws.clear()

    def __len__(self):
        return len(self._ws)


WORKSPACE = _WorkspaceCache()


def reserve_graph_workspace(nbytes, device=None):
    """Before capturing selections into a HIP graph: make sure the graph arena
    can hand out `nbytes` of pre-zeroed workspace on `device` (eager only).
    Size it with the ce_*_workspace_bytes functions, one carve per stream per
    capture."""
    device = torch.device(device if device is not None else "cuda")
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    with torch.cuda.device(device):
        WORKSPACE.arena.reserve(device, int(nbytes))


def committee_view(P, layout="MNC"):
    """(N, M, C, sN, sM, sC, dtype code) of a committee tensor.  'MNC' is the
    reference's stack np.array(pred_prob) (amg_test.py:441); 'NMC' is the
    item-major [N, M, C] tensor.  Any strides are accepted."""
    _on_gpu(P, "committee")
    if P.dim() != 3:
        raise ValueError(f"committee must be 3-D, got shape {tuple(P.shape)}")
    if P.dtype not in _DT:
        raise TypeError(f"committee dtype {P.dtype} not in float32/float64/bfloat16")
    if layout == "MNC":
        M, N, C = P.shape
        sM, sN, sC = P.stride()
    elif layout == "NMC":
        N, M, C = P.shape
        sN, sM, sC = P.stride()
    else:
        raise ValueError(f"layout must be one of {LAYOUTS}, got {layout!r}")
    if M < 1 or C < 1:
        raise ValueError(f"committee needs M >= 1 members and C >= 1 classes, got M={M}, C={C}")
    return N, M, C, sN, sM, sC, _DT[P.dtype]


def committee_entropy(P, layout="MNC", return_mean=False):
    """amg_test.py:441+443 per item: f64 entropies [N] (and the [N, C] mean)."""
    N, M, C, sN, sM, sC, dt = committee_view(P, layout)
    ent = torch.empty(N, dtype=torch.float64, device=P.device)
    mean = torch.empty((N, C), dtype=torch.float64, device=P.device) if return_mean else None
    call("ce_committee_entropy", _p(P), dt, N, M, C, sN, sM, sC, _p(mean), _p(ent), _stream(P.device))
    return (ent, mean) if return_mean else ent


def log_f64(x):
    """glibc's log(x) as the engine evaluates it inside every entropy
    (ce_log_f64; verification against the C library)."""
    _on_gpu(x, "x")
    x = x.contiguous()
    if x.dtype != torch.float64:
        raise ValueError("log_f64 takes float64")
    y = torch.empty_like(x)
    call("ce_log_f64", _p(x), x.numel(), _p(y), _stream(x.device))
    return y


def exp_f64(x):
    """glibc's exp(x) as the engine evaluates it in the GaussianNB member
    (ce_exp_f64; verification against the C library)."""
    _on_gpu(x, "x")
    x = x.contiguous()
    if x.dtype != torch.float64:
        raise ValueError("exp_f64 takes float64")
    y = torch.empty_like(x)
    call("ce_exp_f64", _p(x), x.numel(), _p(y), _stream(x.device))
    return y


def approx_entropy(rows):
    """The single-block pools' approximate entropy of exact consensus rows
    [n, C] f64 (ce_approx_entropy: log2 units, f32) and their special flags
    (verification of the prefilter's error bound)."""
    _on_gpu(rows, "rows")
    rows = rows.contiguous()
    if rows.dtype != torch.float64 or rows.dim() != 2:
        raise ValueError("approx_entropy takes [n, C] float64")
    n, C = rows.shape
    h2 = torch.empty(n, dtype=torch.float32, device=rows.device)
    sp = torch.empty(n, dtype=torch.uint8, device=rows.device)
    call("ce_approx_entropy", _p(rows), n, C, _p(h2), _p(sp), _stream(rows.device))
    return h2, sp.bool()


def wide_approx_entropy(rows, dtype=torch.bfloat16):
    """The wide stream's approximate prefilter entropy (ce_wide_approx_entropy:
    log2 units, f32) of rows [n, C] f64 -- member sums or means, in the register
    layout k_stream_wide2 uses for a ``dtype`` committee -- and their special
    flags (verification of the margin the C5 prefilter skips items by)."""
    _on_gpu(rows, "rows")
    rows = rows.contiguous()
    if rows.dtype != torch.float64 or rows.dim() != 2:
        raise ValueError("wide_approx_entropy takes [n, C] float64")
    n, C = rows.shape
    h2 = torch.empty(n, dtype=torch.float32, device=rows.device)
    sp = torch.empty(n, dtype=torch.uint8, device=rows.device)
    call("ce_wide_approx_entropy", _p(rows), n, C, _DT[dtype], _p(h2), _p(sp), _stream(rows.device))
    return h2, sp.bool()


def row_div_f64(x, s):
    """x / s as the engine divides each consensus row by its sum inside the
    entropy (ce_row_div_f64: one reciprocal per row; verification against
    IEEE division)."""
    _on_gpu(x, "x")
    x = x.contiguous().to(torch.float64)
    s = s.contiguous().to(torch.float64)
    if x.shape != s.shape:
        raise ValueError("x and s must have one shape")
    y = torch.empty_like(x)
    call("ce_row_div_f64", _p(x), _p(s), x.numel(), _p(y), _stream(x.device))
    return y


def vote_table(votes, C=4):
    """amg_test.py:109-117 on int8 votes [N, A] (-1 = missing): (freq [N, C], ent [N])."""
    _on_gpu(votes, "votes")
    if votes.dtype != torch.int8 or votes.dim() != 2:
        raise ValueError("votes must be a 2-D int8 tensor")
    if votes.stride(1) != 1:
        votes = votes.contiguous()
    N, A = votes.shape
    freq = torch.empty((N, C), dtype=torch.float64, device=votes.device)
    ent = torch.empty(N, dtype=torch.float64, device=votes.device)
    call("ce_vote_entropy", _p(votes), N, A, C, votes.stride(0), _p(freq), _p(ent), _stream(votes.device))
    return freq, ent


def va_table(va):
    """amg_test.py:88-117 from raw [N, A, 2] f64 (valence, arousal), NaN = missing."""
    _on_gpu(va, "va")
    if va.dtype != torch.float64 or va.dim() != 3 or va.shape[2] != 2:
        raise ValueError("va must be a [N, A, 2] float64 tensor")
    va = va.contiguous()
    N, A, _ = va.shape
    freq = torch.empty((N, 4), dtype=torch.float64, device=va.device)
    ent = torch.empty(N, dtype=torch.float64, device=va.device)
    call("ce_va_entropy", _p(va), N, A, _p(freq), _p(ent), _stream(va.device))
    return freq, ent


def segment_mean(frames, offsets, perm=None, out=None):
    """amg_test.py:437 groupby(['s_id']).mean() of one member on the device
    (pandas 1.1.5 group_mean: f64 sequential sums in row order, NaN skipped,
    float32 input -> float32-rounded result).  frames [F, C] f32/f64; song n
    owns rows perm[offsets[n]:offsets[n+1]] (or offsets[n]:offsets[n+1]).
    out: optional [N, C] f32/f64 view with unit column stride (e.g. member m of
    a committee stack); default a new tensor of the frames' dtype."""
    _on_gpu(frames, "frames")
    _on_gpu(offsets, "offsets")
    if frames.dim() != 2 or frames.dtype not in (torch.float32, torch.float64):
        raise ValueError("frames must be a 2-D float32/float64 tensor [F, C]")
    if frames.stride(1) != 1:
        frames = frames.contiguous()
    offsets = offsets.to(torch.int64).contiguous()
    F, C = frames.shape
    N = offsets.numel() - 1
    if N < 0:
        raise ValueError("offsets must hold N + 1 entries")
    if perm is not None:
        _on_gpu(perm, "perm")
        perm = perm.to(torch.int64).contiguous()
    if out is None:
        out = torch.empty((N, C), dtype=frames.dtype, device=frames.device)
    if out.dim() != 2 or tuple(out.shape) != (N, C) or out.stride(1) != 1 or out.dtype not in _DT:
        raise ValueError(f"out must be an [N={N}, C={C}] float32/float64 view with unit column stride")
    call("ce_segment_mean", _p(frames), _DT[frames.dtype], F, C, frames.stride(0), _p(perm), _p(offsets), N,
         _p(out), _DT[out.dtype], out.stride(0), _stream(frames.device))
    return out


class _Member(ctypes.Structure):
    """include/ce.h ce_member."""
    _fields_ = [("p", ctypes.c_void_p), ("dtype", ctypes.c_int32), ("song_level", ctypes.c_int32),
                ("ld", ctypes.c_int64)]


def select_frames(members, offsets, q, perm=None, base_idx=0, song_level=None):
    """amg_test.py:426-445 from the members' FRAME-level outputs in one pass
    (ce_select_frames): per member the groupby(['s_id'])
    mean (:437), the member-sequential mean over the stack, the entropy and the
    top-q over songs -- the [M, N, C] stack is never written.  ``members``:
    device tensors [F, C] (frame rows, song n = rows perm[offsets[n]:
    offsets[n+1]] or offsets[n]:offsets[n+1]) or [N, C] (song-level, e.g. the
    CNN member); ``song_level`` overrides the shape rule per member.  Any q:
    q <= 64 in one pass; larger q through the per-song entropies.
    Returns (vals [q], idx [q]) over the N sorted songs."""
    members = list(members)
    if not members:
        raise ValueError("committee has no members")
    _on_gpu(offsets, "offsets")
    offsets = offsets.to(torch.int64).contiguous()
    N = offsets.numel() - 1
    if N < 0:
        raise ValueError("offsets must hold N + 1 entries")
    if perm is not None:
        _on_gpu(perm, "perm")
        perm = perm.to(torch.int64).contiguous()
    q = _check_q(q)
    C = members[0].shape[1]
    for m, t in enumerate(members):
        _on_gpu(t, f"member {m}")
        if t.dim() != 2 or t.shape[1] != C or t.dtype not in (torch.float32, torch.float64):
            raise ValueError(f"member {m} must be a float32/float64 [*, {C}] tensor")
    if song_level is not None and len(song_level) != len(members):
        raise ValueError("song_level needs one flag per member")
    # F (frames): the permutation's length, else the row count of the frame-level
    # members (rows other than N, or flagged frame-level), else one device read
    F = perm.numel() if perm is not None else None
    if F is None:
        fr = {t.shape[0] for m, t in enumerate(members)
              if (not bool(song_level[m]) if song_level is not None else t.shape[0] != N)}
        if len(fr) > 1:
            raise ValueError(f"frame-level members disagree on the frame count: {sorted(fr)}")
        F = fr.pop() if fr else None
    if F is None:  # every member has N rows: only the offsets tell
        F = int(offsets[-1])
    arr = (_Member * len(members))()
    keep = []
    for m, t in enumerate(members):
        if t.stride(1) != 1:
            t = t.contiguous()
        keep.append(t)
        if song_level is not None:
            sl = bool(song_level[m])
        elif t.shape[0] != N:
            sl = False
        else:  # N rows: song-level unless there are exactly N frames too
            sl = F != N
        # the kernel reads row n of a song-level member and rows < F of a frame-level one
        need = N if sl else F
        if t.shape[0] < need:
            raise ValueError(f"member {m} has {t.shape[0]} rows; a {'song' if sl else 'frame'}-level member needs "
                             f">= {need}")
        arr[m] = _Member(t.data_ptr(), _DT[t.dtype], 1 if sl else 0, t.stride(0))
    lib = _lib.load()
    ws = WORKSPACE.get(offsets.device, lib.ce_select_frames_workspace_bytes(N, q), _sort_path(q))
    vals, idx = _outs(q, offsets.device)
    call("ce_select_frames", ctypes.cast(arr, ctypes.c_void_p), len(members), C, _p(offsets), _p(perm), N, q,
         int(base_idx), _p(ws), ws.numel(), _p(vals), _p(idx), _stream(offsets.device))
    return vals, idx


def _f64_dev(t, device, what):
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(t)
    t = t.to(device=device, dtype=torch.float64)
    return t.contiguous()


def gnb_predict_proba(X, theta, var, class_prior, out=None):
    """GaussianNB(...).predict_proba(X) on the device (sklearn 0.24.1 math,
    deam_classifier.py:211; amg_test.py:435).  X [F, D] f64 frames; theta /
    var [C, D] (theta_, var_ -- sigma_ in 0.24), class_prior [C]."""
    _on_gpu(X, "X")
    if X.dim() != 2 or X.dtype != torch.float64 or X.stride(1) != 1:
        raise ValueError("X must be a float64 [F, D] tensor with unit column stride")
    F, D = X.shape
    theta = _f64_dev(theta, X.device, "theta")
    var = _f64_dev(var, X.device, "var")
    C = theta.shape[0]
    if tuple(theta.shape) != (C, D) or tuple(var.shape) != (C, D):
        raise ValueError(f"theta/var must be [C, {D}]")
    # np.log(class_prior_[i]) (sklearn 0.24.1 _joint_log_likelihood) with the C
    # library's log, as numpy 1.19.5 evaluates it: a device prior through the
    # restated glibc log (ce_log_f64: no host sync, graph-capturable), a host
    # prior through the C library itself
    if isinstance(class_prior, torch.Tensor) and class_prior.device == X.device:
        log_prior = log_f64(class_prior.to(torch.float64).reshape(-1).contiguous())
    else:
        prior = np.asarray(class_prior.cpu() if isinstance(class_prior, torch.Tensor) else class_prior, np.float64)
        log_prior = torch.tensor([math.log(float(p)) if p > 0 else (-math.inf if p == 0 else math.nan)
                                  for p in prior.reshape(-1)], dtype=torch.float64, device=X.device)
    if out is None:
        out = torch.empty((F, C), dtype=torch.float64, device=X.device)
    call("ce_gnb_predict_proba", _p(X), F, D, X.stride(0), _p(theta), _p(var), _p(log_prior), C, _p(out),
         out.stride(0), _stream(X.device))
    return out


def sgd_predict_proba(X, coef, intercept, out=None):
    """SGDClassifier(loss='log').predict_proba(X) on the device (sklearn
    _predict_proba_lr, deam_classifier.py:214; amg_test.py:435).  coef [K, D],
    intercept [K]; K = C (OvR) or 1 (binary, C = 2)."""
    _on_gpu(X, "X")
    if X.dim() != 2 or X.dtype != torch.float64 or X.stride(1) != 1:
        raise ValueError("X must be a float64 [F, D] tensor with unit column stride")
    F, D = X.shape
    coef = _f64_dev(coef, X.device, "coef")
    if coef.dim() == 1:
        coef = coef.unsqueeze(0)
    K = coef.shape[0]
    intercept = _f64_dev(intercept, X.device, "intercept").reshape(-1)
    C = 2 if K == 1 else K
    if coef.shape[1] != D or intercept.numel() != K:
        raise ValueError(f"coef must be [K, {D}] and intercept [K]")
    if out is None:
        out = torch.empty((F, C), dtype=torch.float64, device=X.device)
    call("ce_sgd_predict_proba", _p(X), F, D, X.stride(0), _p(coef), _p(intercept), K, C, _p(out),
         out.stride(0), _stream(X.device))
    return out


def xgb_predict_proba(X, forest, out=None, out_dtype=torch.float32):
    """XGBClassifier(...).predict_proba(X) on the device (xgboost 1.3.3
    predictor restated in csrc/ce_xgb.hip; xgboost/sklearn.py:991-1029,
    amg_test.py:435).  X [F, D] f32/f64 frames (cast to float32 like DMatrix,
    NaN = missing); ``forest`` an ``ce_amd.xgb.XgbForest`` (or its JSON).
    Returns [F, C] ``out_dtype`` (float32 = what xgboost returns; float64 = its
    exact upcast, ready for a committee stack)."""
    from .xgb import XgbForest

    _on_gpu(X, "X")
    if X.dim() != 2 or X.dtype not in (torch.float32, torch.float64) or X.stride(1) != 1:
        raise ValueError("X must be a float32/float64 [F, D] tensor with unit column stride")
    if not isinstance(forest, XgbForest):
        forest = XgbForest.from_json(forest)
    F, D = X.shape
    if forest.max_feature() >= D:
        raise ValueError(f"the forest splits on feature {forest.max_feature()} but X has {D} columns")
    G, C = forest.n_groups, forest.n_classes
    if out is None:
        out = torch.empty((F, C), dtype=out_dtype, device=X.device)
    if out.dim() != 2 or out.shape[0] != F or out.shape[1] < C or out.stride(1) != 1 or out.dtype not in _DT:
        raise ValueError(f"out must be a float [{F}, >={C}] tensor with unit column stride")
    nodes, leaves, goff, depth = forest.device_arrays(X.device)
    if depth <= LANE_TABLE_DEPTH:  # the reference's max_depth=5: prebuilt per-tree lane tables
        table = forest.lane_table(X.device, D)
        call("ce_xgb_predict_proba_lanes", _p(X), _DT[X.dtype], F, D, X.stride(0), _p(table), table.shape[1],
             _p(goff), G, depth, float(forest.base_margin), C, _p(out), _DT[out.dtype], out.stride(0),
             _stream(X.device))
    else:
        call("ce_xgb_predict_proba", _p(X), _DT[X.dtype], F, D, X.stride(0), _p(nodes), _p(leaves), _p(goff), G,
             depth, float(forest.base_margin), C, _p(out), _DT[out.dtype], out.stride(0), _stream(X.device))
    return out


LANE_TABLE_DEPTH = 5  # csrc/ce_xgb.hip kXgbLaneDepth: 2^(d+1) heap entries fit one wave


def _check_q(q):
    """Any q >= 0, as the reference's -q (amg_test.py:547-553).  Outputs hold q
    slots (padding -- val NaN, idx -1 -- past the pool); q <= CE_MAX_Q runs on
    the list kernels, larger q on the sort path (workspace grows with N)."""
    q = int(q)
    if q < 0:
        raise ValueError(f"q={q} is negative")
    if q > _Q_ABI_MAX:  # every entry point takes q as int32 (ctypes would truncate it silently)
        raise ValueError(f"q={q} exceeds the C-ABI's int32 q; clamp it to the pool size (min(q, N)) first")
    return q


_Q_ABI_MAX = 2**31 - 1


def _sort_path(q):
    """q > CE_MAX_Q runs on the sort path: its workspace is per call (see _WorkspaceCache)."""
    return q > _lib.CE_MAX_Q


def _outs(q, device, lead=()):
    return (torch.empty(lead + (q,), dtype=torch.float64, device=device),
            torch.empty(lead + (q,), dtype=torch.int64, device=device))


def topq(ent, q, base_idx=0):
    """np.argsort(ent)[::-1][:q] under the total order (NaN first, desc, lowest
    index).  Returns (vals [q], idx [q]); idx = -1 marks empty slots."""
    _on_gpu(ent, "ent")
    q = _check_q(q)
    ent = ent.contiguous().to(torch.float64)
    N = ent.numel()
    lib = _lib.load()
    ws = WORKSPACE.get(ent.device, lib.ce_topq_workspace_bytes(N, q), _sort_path(q))
    vals, idx = _outs(q, ent.device)
    call("ce_topq", _p(ent), N, q, int(base_idx), _p(ws), ws.numel(), _p(vals), _p(idx), _stream(ent.device))
    return vals, idx


def topq_merge(vals, idx, q):
    """Merge best-first candidate lists of q slots each (e.g. per-GPU top-q
    after an all-gather) into the global top-q."""
    _on_gpu(vals, "vals")
    q = _check_q(q)
    vals = vals.contiguous().view(-1)
    idx = idx.contiguous().view(-1)
    if q == 0:
        return _outs(0, vals.device)
    if vals.numel() != idx.numel() or vals.numel() == 0 or vals.numel() % q:
        raise ValueError("vals/idx must hold nlists * q entries")
    ov, oi = _outs(q, vals.device)
    call("ce_topq_merge", _p(vals), _p(idx), vals.numel() // q, q, _p(ov), _p(oi), _stream(vals.device))
    return ov, oi


def select_mc(P, q, layout="MNC", base_idx=0, excl=None):
    """Fused amg_test.py:441-445: (vals [q], idx [q]) best-first.  excl: an
    optional exclusion bitmap (int32 [ceil(N/32)], bit i set = item i is out
    of the pool), see excl_bitmap / mark_selected."""
    N, M, C, sN, sM, sC, dt = committee_view(P, layout)
    q = _check_q(q)
    lib = _lib.load()
    ws = WORKSPACE.get(P.device, lib.ce_select_mc_workspace_bytes(N, q), _sort_path(q))
    vals, idx = _outs(q, P.device)
    if excl is None:
        call("ce_select_mc", _p(P), dt, N, M, C, sN, sM, sC, q, int(base_idx), _p(ws), ws.numel(), _p(vals),
             _p(idx), _stream(P.device))
    else:
        _check_excl(excl, N)
        call("ce_select_mc_excl", _p(P), dt, N, M, C, sN, sM, sC, _p(excl), q, int(base_idx), _p(ws), ws.numel(),
             _p(vals), _p(idx), _stream(P.device))
    return vals, idx


def excl_bitmap(n, device=None):
    """An all-clear exclusion bitmap for n items (int32 words on the device)."""
    words = _lib.load().ce_excl_words(int(n))
    return torch.zeros(max(int(words), 1), dtype=torch.int32, device=device)


def _check_excl(excl, n):
    _on_gpu(excl, "excl")
    if excl.dtype != torch.int32 or not excl.is_contiguous() or excl.numel() * 32 < n:
        raise ValueError(f"excl must be a contiguous int32 bitmap of >= {(n + 31) // 32} words")


def mark_selected(excl, n, idx, base_idx=0):
    """Set the bitmap bits of the selected positions idx (device int64; -1
    slots ignored) -- stream-ordered after the selection that produced them."""
    _check_excl(excl, n)
    _on_gpu(idx, "idx")
    idx = idx.to(torch.int64).contiguous()
    call("ce_mark_selected", _p(excl), int(n), _p(idx), idx.numel(), int(base_idx), _stream(excl.device))


class MCPlan:
    """Pre-bound mc selection with its own workspace and outputs: what the
    bench and the multi-GPU driver launch every step.  step() / step_cands()
    run the whole selection in one launch; partial() + finish() /
    finish_cands() are the two stages as separate launches."""

    def __init__(self, P, q, layout="NMC", base_idx=0):
        self.P = P
        self.N, self.M, self.C, self.sN, self.sM, self.sC, self.dt = committee_view(P, layout)
        self.q = _check_q(q)
        self.base_idx = int(base_idx)
        lib = _lib.load()
        self.ws_bytes = lib.ce_select_mc_workspace_bytes(self.N, self.q)
        self.ws = new_workspace(self.ws_bytes, P.device)
        self.vals, self.idx = _outs(self.q, P.device)

    def partial(self):
        call("ce_select_mc_partial", _p(self.P), self.dt, self.N, self.M, self.C, self.sN, self.sM, self.sC, self.q,
             self.base_idx, _p(self.ws), self.ws_bytes, _stream(self.P.device))

    def finish(self):
        call("ce_select_finish", self.N, self.q, _p(self.ws), self.ws_bytes, _p(self.vals), _p(self.idx),
             _stream(self.P.device))
        return self.vals, self.idx

    def finish_cands(self, out=None):
        """Stage 2 writing this pool's q candidate records (ce_cand: order key,
        position; as an int64 [q, 2] tensor) -- the all-gather send buffer of
        the multi-GPU merge.  partial() / finish*() need q <= CE_MAX_Q."""
        if out is None:
            out = torch.empty((self.q, 2), dtype=torch.int64, device=self.P.device)
        call("ce_select_finish_cands", self.N, self.q, _p(self.ws), self.ws_bytes, _p(out), _stream(self.P.device))
        return out

    def step(self):
        """The whole selection (ce_select_mc; ONE launch for q <= 64: stage 2
        folded into stage 1's last block): (vals [q], idx [q])."""
        call("ce_select_mc", _p(self.P), self.dt, self.N, self.M, self.C, self.sN, self.sM, self.sC, self.q,
             self.base_idx, _p(self.ws), self.ws_bytes, _p(self.vals), _p(self.idx), _stream(self.P.device))
        return self.vals, self.idx

    def step_cands(self, out=None):
        """This pool's q candidate records (int64 [q, 2], the multi-GPU send
        buffer; ce_select_mc_cands, ONE launch for q <= 64)."""
        if out is None:
            out = torch.empty((self.q, 2), dtype=torch.int64, device=self.P.device)
        call("ce_select_mc_cands", _p(self.P), self.dt, self.N, self.M, self.C, self.sN, self.sM, self.sC, self.q,
             self.base_idx, _p(self.ws), self.ws_bytes, _p(out), _stream(self.P.device))
        return out

    def __call__(self):
        return self.step()


def merge_cands(cands, q):
    """Merge nlists lists of q candidate records (int64 [nlists*q, 2] or
    [nlists, q, 2], each list best-first -- e.g. the all-gather receive buffer)
    into the final (vals [q], idx [q])."""
    _on_gpu(cands, "cands")
    q = _check_q(q)
    if cands.dtype != torch.int64 or cands.shape[-1] != 2 or not cands.is_contiguous():
        raise ValueError("cands must be a contiguous int64 [..., 2] tensor of records")
    n = cands.numel() // 2
    if q == 0 or n == 0 or n % q:
        if q == 0:
            return _outs(0, cands.device)
        raise ValueError("cands must hold nlists * q records")
    ov, oi = _outs(q, cands.device)
    call("ce_merge_cands", _p(cands), n // q, q, _p(ov), _p(oi), _stream(cands.device))
    return ov, oi


class MCChunkJob:
    """amg_test.py:441-445 over a pool larger than HBM (BASELINE configs[4]),
    streamed as consecutive chunks: ``add(P_chunk)`` scores one resident chunk
    (pool positions continue from the previous chunk) and folds its top-q into
    a running list of q candidate records on the device; ``result()`` is the
    selection over everything added -- identical to select_mc on the whole
    pool, ties included (any q)."""

    def __init__(self, q, layout="NMC", device=None):
        self.q = _check_q(q)
        self.layout = layout
        self.device = torch.device(device) if device is not None else None
        self.running = None
        self.n_items = 0
        self._fresh = True
        self._ranges = []  # [lo, hi) position ranges added so far

    def add(self, P, base_idx=None):
        """Score chunk P (layout as constructed); its items are pool positions
        base_idx .. base_idx + N - 1 (default: right after the previous chunk)."""
        N, M, C, sN, sM, sC, dt = committee_view(P, self.layout)
        if self.running is None:
            if self.device is not None and self.device.index is not None and P.device != self.device:
                raise ValueError(f"chunk on {P.device}, job on {self.device}")
            self.running = torch.empty((self.q, 2), dtype=torch.int64, device=P.device)
        elif P.device != self.running.device:
            raise ValueError(f"chunk on {P.device}, but the job's running list lives on {self.running.device}")
        base = self.n_items if base_idx is None else int(base_idx)
        if base < 0:
            raise ValueError(f"base_idx must be >= 0, got {base}")
        for lo, hi in self._ranges:  # a position scored twice would be merged silently
            if base < hi and lo < base + N:
                raise ValueError(f"chunk positions [{base}, {base + N}) overlap an added chunk [{lo}, {hi})")
        if N > 0:
            self._ranges.append((base, base + N))
        lib = _lib.load()
        ws = WORKSPACE.get(P.device, lib.ce_select_mc_chunk_workspace_bytes(N, self.q), _sort_path(self.q))
        first = 1 if self._fresh else 0
        call("ce_select_mc_chunk", _p(P), dt, N, M, C, sN, sM, sC, self.q, base, _p(self.running), first, _p(ws),
             ws.numel(), _stream(P.device))
        self._fresh = False
        self.n_items = max(self.n_items, base + N)
        return self

    def running_records(self, device=None):
        """The running list: q candidate records (int64 [q, 2], best first; an
        empty list -- key 0, idx -1 -- when no chunk was added), e.g. the send
        buffer of the multi-GPU all-gather."""
        if self.running is None:
            dev = device if device is not None else (self.device or torch.device("cuda", torch.cuda.current_device()))
            empty = torch.zeros((self.q, 2), dtype=torch.int64, device=dev)
            empty[:, 1] = -1
            return empty
        return self.running

    def result(self):
        """(vals [q], idx [q]) best-first over every chunk added (idx -1 padding)."""
        if self.running is None:
            raise ValueError("no chunk added")
        return merge_cands(self.running, self.q)


def select_mc_chunks(chunks, q, layout="NMC"):
    """Convenience over MCChunkJob: ``chunks`` yields consecutive device tensors
    (or (tensor, base_idx) pairs) of one pool."""
    job = None
    for ch in chunks:
        P, base = ch if isinstance(ch, tuple) else (ch, None)
        if job is None:
            job = MCChunkJob(q, layout, P.device)
        job.add(P, base)
    if job is None:
        raise ValueError("no chunks")
    return job.result()


def select_mix(P, hc, q, layout="MNC"):
    """Fused amg_test.py:473-480: top-q over the row stack [mc (N); hc (N_h)]."""
    N, M, C, sN, sM, sC, dt = committee_view(P, layout)
    _on_gpu(hc, "hc table")
    if hc.dim() != 2 or hc.shape[1] != C:
        raise ValueError(f"hc table must be [N_h, {C}]")
    hc = hc.to(torch.float64)
    if hc.stride(1) != 1:
        hc = hc.contiguous()
    q = _check_q(q)
    N_h = hc.shape[0]
    lib = _lib.load()
    ws = WORKSPACE.get(P.device, lib.ce_select_mix_workspace_bytes(N, N_h, q), _sort_path(q))
    vals, idx = _outs(q, P.device)
    call("ce_select_mix", _p(P), dt, N, M, C, sN, sM, sC, _p(hc), N_h, hc.stride(0), q, _p(ws), ws.numel(),
         _p(vals), _p(idx), _stream(P.device))
    return vals, idx


def select_batched(P, offsets, q, layout="MNC"):
    """U users in one launch; user u owns items offsets[u]:offsets[u+1].
    Returns (vals [U, q], idx [U, q]) with user-local positions."""
    N, M, C, sN, sM, sC, dt = committee_view(P, layout)
    _on_gpu(offsets, "offsets")
    offsets = offsets.to(torch.int64).contiguous()
    U = offsets.numel() - 1
    if U < 1:
        raise ValueError("offsets must hold U + 1 >= 2 entries")
    q = _check_q(q)
    lib = _lib.load()
    ws = WORKSPACE.get(P.device, lib.ce_select_batched_workspace_bytes(N, U, q), _sort_path(q))
    vals, idx = _outs(q, P.device, (U,))
    call("ce_select_batched", _p(P), dt, N, M, C, sN, sM, sC, _p(offsets), U, q, _p(ws), ws.numel(), _p(vals),
         _p(idx), _stream(P.device))
    return vals, idx
