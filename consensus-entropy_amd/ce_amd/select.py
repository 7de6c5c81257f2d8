"""Drop-in query selection for AMG_Tester.run (amg_test.py:425-489).

``select_queries`` is the function-level seam: it takes exactly what the
reference has in hand at that point (the list ``pred_prob`` of per-member
[N, C] probability frames, the human-consensus frame, the unlabeled pool ids)
and returns what the reference computes (positions ``q_ind`` -- or, for
``rand``, the ids ``q_songs``).  ``ConsensusEntropySelector`` wraps it with the
reference's per-epoch bookkeeping (index -> song id mapping, shrinking the hc
pool).  All arithmetic runs in the HIP kernels; inputs given as numpy/pandas
are uploaded, results are copied back.

Semantics kept from the reference:
  mc   amg_test.py:441-447  mean over members, entropy, top-q, ids from the
                            LAST member frame's index
  hc   amg_test.py:451-455  entropy of the remaining hc rows, top-q, drop them
  mix  amg_test.py:473-484  ROW stack [mc; hc] (not a blend), top-q over the
                            union, may pick one song twice, drop picks from hc
  rand amg_test.py:486-489  np.random.shuffle of the unique pool ids (global
                            legacy RNG unless an rng is passed), first q
Tie order: the reference's argsort has none; here NaN first, then entropy
descending, then lowest position.
Errors: ValueError for a bad mode or shapes (the CLI keeps the reference's
print-and-exit at amg_test.py:577-579).
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops

MODES = ("mc", "hc", "mix", "rand")


def _device(device):
    if device is None:
        if not torch.cuda.is_available():
            raise RuntimeError("ce_amd needs a HIP device (MI355X); there is no CPU path")
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


def stack_committee(committee, device=None, layout="MNC"):
    """The committee as one device tensor.  A list of M [N, C] members is
    stacked like np.array(pred_prob) (amg_test.py:441): mixed float32/float64
    members are upcast to float64 exactly as numpy does; all-float32 (or
    all-bfloat16) members stay narrow -- the kernel accumulates in float64
    either way."""
    dev = _device(device)
    if isinstance(committee, torch.Tensor):
        return committee.to(dev), layout
    if isinstance(committee, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(committee)).to(dev), layout
    members = list(committee)
    if not members:
        raise ValueError("committee has no members")
    if all(isinstance(m, torch.Tensor) for m in members):
        dts = {m.dtype for m in members}
        dt = members[0].dtype if len(dts) == 1 else torch.float64
        return torch.stack([m.to(dev, dt) for m in members]), "MNC"
    arrs = [np.asarray(getattr(m, "values", m)) for m in members]
    shapes = {a.shape for a in arrs}
    if len(shapes) != 1:
        raise ValueError(f"committee members disagree on shape: {sorted(shapes)}")
    dt = np.result_type(*arrs)
    if dt not in (np.float32, np.float64):
        dt = np.float64
    return torch.from_numpy(np.stack(arrs).astype(dt, copy=False)).to(dev), "MNC"


def song_groups(s_id):
    """Host geometry of groupby(['s_id']) (sort=True): the sorted unique song
    ids, CSR offsets of each song's frames, and the stable permutation that
    groups the frames (None when they already are, in sorted order)."""
    ids = np.asarray(getattr(s_id, "values", s_id))
    uniq, labels = np.unique(ids, return_inverse=True)
    labels = labels.reshape(-1)
    offsets = np.concatenate([[0], np.cumsum(np.bincount(labels, minlength=len(uniq)))]).astype(np.int64)
    perm = None if np.all(labels[1:] >= labels[:-1]) else np.argsort(labels, kind="stable").astype(np.int64)
    return uniq, offsets, perm


def committee_from_frames(members, s_id, device=None):
    """The committee stack np.array(pred_prob) of amg_test.py:426-441, built on
    the device.  `members` in mod_list order; each is either a frame-level
    predict_proba array [F, C] (rows in X_train order, grouped by `s_id` with
    the segment-mean kernel, :437) or an already song-level [N, C] frame/array
    (the CNN member, :432-433, taken positionally as np.array does).  Returns
    (stack [M, N, C] on the device, the sorted song ids of the groupby rows).
    The stack is float64 unless every member is float32 (np.array's rule)."""
    dev = _device(device)
    uniq, offsets, perm = song_groups(s_id)
    N = len(uniq)
    F = len(np.asarray(getattr(s_id, "values", s_id)))
    # members: device tensors (e.g. ops.gnb_predict_proba outputs) stay on the device
    arrs = [m if isinstance(m, torch.Tensor) else np.asarray(getattr(m, "values", m)) for m in members]
    if not arrs:
        raise ValueError("committee has no members")
    C = arrs[0].shape[1]
    f32 = [a.dtype in (np.float32, torch.float32) for a in arrs]
    dt = torch.float32 if all(f32) else torch.float64
    stack = torch.empty((len(arrs), N, C), dtype=dt, device=dev)
    offs_d = torch.from_numpy(offsets).to(dev)
    perm_d = torch.from_numpy(perm).to(dev) if perm is not None else None
    for m, a in enumerate(arrs):
        if a.ndim != 2 or a.shape[1] != C:
            raise ValueError(f"member {m} has shape {tuple(a.shape)}, expected [*, {C}]")
        if isinstance(a, torch.Tensor):
            t = a.to(dev)
            if t.dtype not in (torch.float32, torch.float64):
                t = t.to(torch.float64)
        else:
            t = None
        if a.shape[0] == F and (F != N or perm is not None):  # frame-level: groupby mean on the device
            if t is None:
                t = torch.from_numpy(np.ascontiguousarray(a, dtype=a.dtype if a.dtype in (np.float32, np.float64)
                                                          else np.float64)).to(dev)
            ops.segment_mean(t.contiguous(), offs_d, perm_d, out=stack[m])
        elif a.shape[0] == N:  # song-level member
            stack[m] = (t if t is not None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)).to(dt)
        else:
            raise ValueError(f"member {m} has {a.shape[0]} rows: neither {F} frames nor {N} songs")
    return stack, uniq


def select_from_frames(members, s_id, q, device=None):
    """amg_test.py:426-447 in ONE kernel from the members' frame-level outputs
    (ops.select_frames): `members` in mod_list order, each a
    frame-level predict_proba [F, C] (rows in X_train order, song ids `s_id`)
    or a song-level [N, C] member (the CNN, :430-433); the [M, N, C] stack is
    never built.  Returns (q_ind positions over the sorted songs, the sorted
    song ids) -- q_songs = ids[q_ind] as :447 maps them."""
    dev = _device(device)
    uniq, offsets, perm = song_groups(s_id)
    N, F = len(uniq), len(np.asarray(getattr(s_id, "values", s_id)))
    ts, sl = [], []
    for m, a in enumerate(members):
        t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(getattr(a, "values", a)))
        if t.dtype not in (torch.float32, torch.float64):
            t = t.to(torch.float64)
        if t.dim() != 2 or t.shape[0] not in (F, N):
            raise ValueError(f"member {m} has shape {tuple(t.shape)}: neither {F} frames nor {N} songs")
        ts.append(t.to(dev))
        sl.append(not (t.shape[0] == F and (F != N or perm is not None)))  # committee_from_frames' rule
    offs = torch.from_numpy(offsets).to(dev)
    pd_ = torch.from_numpy(perm).to(dev) if perm is not None else None
    _, idx = ops.select_frames(ts, offs, q, perm=pd_, song_level=sl)
    return _positions(idx), uniq


def _hc_tensor(hc, votes, C, dev):
    if hc is not None:
        arr = np.asarray(getattr(hc, "values", hc), dtype=np.float64) if not isinstance(hc, torch.Tensor) else hc
        t = torch.as_tensor(arr, dtype=torch.float64).to(dev)
        if t.dim() != 2:
            raise ValueError("hc table must be 2-D [N_h, C]")
        return t
    if votes is not None:
        v = torch.as_tensor(np.asarray(votes, dtype=np.int8) if not isinstance(votes, torch.Tensor) else votes)
        freq, _ = ops.vote_table(v.to(dev), C=C)
        return freq
    raise ValueError("hc/mix modes need `hc` (frequency table) or `votes`")


def _positions(idx):
    i = idx.cpu().numpy()
    return i[i >= 0]


def select_queries(mode, q, *, committee=None, hc=None, votes=None, pool=None, rng=None, layout="MNC",
                   device=None, n_classes=4):
    """One selection step of amg_test.py:425-489.

    mode       'mc' | 'hc' | 'mix' | 'rand'
    q          number of queries (self.queries)
    committee  list of M [N, C] member arrays/frames (pred_prob), or a stacked
               array/tensor in `layout` ('MNC' = [M, N, C], 'NMC' = [N, M, C])
    hc         [N_h, C] human-consensus frequency table (this_consensus_hc)
    votes      alternatively, int8 votes [N_h, A] (-1 = missing) -> hc table
    pool       rand mode: the unlabeled pool ids (X_train.index)
    rng        rand mode: np.random.RandomState (default: the global legacy RNG)
    Returns positions (np.int64) for mc/hc/mix -- mix positions index the
    stack [mc rows; hc rows] -- and the chosen ids (list) for rand.
    """
    if mode not in MODES:
        raise ValueError(f"mode must be one of {MODES}, got {mode!r}")
    q = int(q)
    if q < 0:  # any other q is the reference's -q (amg_test.py:547-553): argsort[::-1][:q] keeps min(q, N)
        raise ValueError(f"q = {q} is negative")
    if mode == "rand":
        if pool is None:
            raise ValueError("rand mode needs `pool`")
        pos_songs = list(dict.fromkeys(getattr(pool, "tolist", lambda: list(pool))()))  # .unique().tolist()
        (rng if rng is not None else np.random).shuffle(pos_songs)
        return pos_songs[:q]
    dev = _device(device)
    if mode == "mc":
        if committee is None:
            raise ValueError("mc mode needs `committee`")
        P, lay = stack_committee(committee, dev, layout)
        _, idx = ops.select_mc(P, min(q, _items(P, lay)), lay)
        return _positions(idx)
    if mode == "hc":
        H = _hc_tensor(hc, votes, n_classes, dev)
        P = H.unsqueeze(1)  # [N_h, M=1, C]: mean over one member is the row itself
        _, idx = ops.select_mc(P, min(q, H.shape[0]), "NMC")
        return _positions(idx)
    # mix
    if committee is None:
        raise ValueError("mix mode needs `committee`")
    P, lay = stack_committee(committee, dev, layout)
    H = _hc_tensor(hc, votes, n_classes, dev)
    _, idx = ops.select_mix(P, H, min(q, _items(P, lay) + H.shape[0]), lay)
    return _positions(idx)


def _items(P, layout):
    """Pool items of a committee tensor: no more than these can be selected
    (the ops outputs hold q slots; argsort[::-1][:q] returns min(q, N))."""
    return P.shape[1] if layout == "MNC" else P.shape[0]


class ConsensusEntropySelector:
    """The selection branch of AMG_Tester.run per epoch (amg_test.py:425-489),
    including the id mapping and the hc-pool shrinking the reference does
    inline.  Pool removal from X_train/id_tr (:521-531) stays with the caller,
    as in the reference.

        sel = ConsensusEntropySelector(queries=10, mode="mix")
        q_songs, this_consensus_hc = sel.select(pred_prob=frames, consensus_hc=hc_frame)
    """

    def __init__(self, queries, mode, rng=None, device=None):
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}, got {mode!r}")
        self.queries = int(queries)
        self.mode = mode
        self.rng = rng
        self.device = device

    def select(self, pred_prob=None, consensus_hc=None, pool_ids=None):
        """Returns (q_songs, consensus_hc after removal)."""
        mode, q = self.mode, self.queries
        if mode == "rand":
            return select_queries("rand", q, pool=pool_ids, rng=self.rng), consensus_hc
        if mode in ("mc", "mix"):
            if pred_prob is None or len(pred_prob) == 0:
                raise ValueError(f"{mode} mode needs pred_prob")
            last_index = list(getattr(pred_prob[-1], "index", range(len(pred_prob[-1]))))
        if mode == "mc":
            q_ind = select_queries("mc", q, committee=pred_prob, device=self.device)
            return [last_index[i] for i in q_ind], consensus_hc
        hc_index = list(getattr(consensus_hc, "index", range(len(consensus_hc))))
        if mode == "hc":
            q_ind = select_queries("hc", q, hc=consensus_hc, device=self.device)
            q_songs = [hc_index[i] for i in q_ind]
        else:  # mix: positions index [mc rows (last member's index); hc rows]
            q_ind = select_queries("mix", q, committee=pred_prob, hc=consensus_hc, device=self.device)
            n = len(last_index)
            q_songs = [last_index[i] if i < n else hc_index[i - n] for i in q_ind]
        return q_songs, _drop_rows(consensus_hc, q_songs)


def _drop_rows(hc, q_songs):
    """this_consensus_hc[~this_consensus_hc.index.isin(q_songs)] (amg_test.py:455, :484)."""
    if hasattr(hc, "index") and hasattr(hc.index, "isin"):
        return hc[~hc.index.isin(q_songs)]
    keep = [i for i in range(len(hc)) if i not in set(q_songs)]
    return np.asarray(hc)[keep]
