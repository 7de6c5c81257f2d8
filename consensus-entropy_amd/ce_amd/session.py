"""Device-resident multi-epoch selection.

The reference shrinks its pools on the host every epoch: the queried songs
leave X_train / id_tr (amg_test.py:521-531) and the hc frame
(``this_consensus_hc[~index.isin(q_songs)]``, :455, :484), and the next epoch's
``pred_prob`` is computed over what is left.  A ``SelectionSession`` keeps the
FULL pool on the device instead, with one exclusion bitmap per pool: each
epoch the caller hands in the committee's probabilities over the full pool
(e.g. from on-device member inference), the engine selects among the items
whose bit is clear, and marks the picks -- no pool bookkeeping crosses PCIe,
only the q picked positions come back.

Positions returned are positions in the FULL pool (stable across epochs), so
the caller maps them to song ids once.  Selection per epoch equals the
reference's on the shrunken pool (tests/test_gpu_parity.py::test_session_*).

Modes (amg_test.py:425-489):
  mc    committee over the full pool [M, N, C] (or [N, M, C]), excluding queried items
  hc    the human-consensus table, fixed at construction, excluding queried rows
  mix   both.  The hc table keeps the reference's OWN row order (annotation
        order, :359/:376), not the committee's (sorted s_id, :437), so the
        lowest-position tie-break inside the hc segment of [mc; hc] (:477) is
        the reference's; ``hc_to_mc[j]`` names the committee item of hc row j
        (-1: the song is not in the committee's pool).  A pick through either
        part removes the song from both, as :484 + :521-531 do by id.
        Positions: i in [0, N) = committee item i, N + j = hc row j (the row
        stack [mc; hc] of select_queries, over the full pools)
  rand  amg_test.py:486-489: ``pos_songs = X_train.index.unique().tolist();
        np.random.shuffle(pos_songs); pos_songs[:q]`` -- the legacy shuffle of
        the REMAINING songs in the order they first appear in X_train.
        ``rand_order`` gives that order as positions (the pool position of the
        first song of X_train, of the second, ...); the remaining songs keep it
        as the pool shrinks (a DataFrame drop keeps row order), so with the
        caller's RandomState (or the global one the reference seeds with
        np.random.seed(1987), :55) the picks are the reference's, draw for
        draw.  Default: ascending positions, i.e. X_train's songs appear in
        position order.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from .select import MODES, _device, _hc_tensor, stack_committee


class SelectionSession:
    def __init__(self, queries, mode, n_items, *, hc=None, votes=None, hc_to_mc=None, rng=None, device=None,
                 n_classes=4, rand_order=None):
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}, got {mode!r}")
        self.q = int(queries)
        if self.q < 0:  # any other q, as the reference's -q (amg_test.py:547-553)
            raise ValueError(f"queries = {self.q} is negative")
        self.mode = mode
        self.N = int(n_items)
        self.dev = _device(device)
        self.rng = rng
        self.H = None
        if mode in ("hc", "mix"):
            self.H = _hc_tensor(hc, votes, n_classes, self.dev).to(torch.float64).contiguous()
            if mode == "hc":
                self.N = self.H.shape[0]
        self.excl = ops.excl_bitmap(self.N, self.dev)
        self.n_selected = 0
        self.rand_order = None
        if mode == "rand":
            order = np.arange(self.N) if rand_order is None else np.asarray(rand_order, dtype=np.int64).reshape(-1)
            if order.shape[0] != self.N or not np.array_equal(np.sort(order), np.arange(self.N)):
                raise ValueError("rand_order must be a permutation of the n_items pool positions")
            self.rand_order = order
        if mode == "mix":
            Nh = self.H.shape[0]
            if hc_to_mc is None:
                if Nh != self.N:
                    raise ValueError("mix: pass hc_to_mc (committee item of each hc row) when the pools differ")
                hc_to_mc = np.arange(Nh)
            h2m = np.asarray(hc_to_mc, dtype=np.int64).reshape(-1)
            if h2m.shape[0] != Nh or (h2m >= self.N).any() or (h2m < -1).any():
                raise ValueError("hc_to_mc must give, per hc row, a committee item in [0, n_items) or -1")
            valid = h2m[h2m >= 0]
            if len(np.unique(valid)) != len(valid):
                raise ValueError("hc_to_mc maps two hc rows to one committee item")
            m2h = np.full(self.N, -1, np.int64)
            m2h[valid] = np.flatnonzero(h2m >= 0)
            self.h2m = torch.from_numpy(h2m).to(self.dev)
            self.m2h = torch.from_numpy(m2h).to(self.dev)
            self.Nh = Nh
            self.excl_hc = ops.excl_bitmap(Nh, self.dev)

    @property
    def remaining(self):
        return self.N - self.n_selected

    def _mc(self, committee, layout, q):
        P, lay = stack_committee(committee, self.dev, layout)
        n = P.shape[1] if lay == "MNC" else P.shape[0]
        if n != self.N:
            raise ValueError(f"committee covers {n} items, the session's pool has {self.N}")
        return ops.select_mc(P, q, lay, excl=self.excl)

    def _hc(self, q, excl=None):
        return ops.select_mc(self.H.unsqueeze(1), q, "NMC", excl=self.excl if excl is None else excl)

    def _slots(self):
        """Output slots per part: q, but never more than the pools hold (argsort
        [::-1][:q] returns min(q, N)), so a huge q costs no huge buffers."""
        n = self.N + (self.Nh if self.mode == "mix" else 0)
        return min(self.q, n)

    def select(self, committee=None, layout="MNC"):
        """One epoch: returns the q picked positions (np.int64; fewer when the
        pool runs dry) and removes them from the pool."""
        q = self.q
        if self.mode == "rand":  # amg_test.py:487-489 over the remaining songs, in X_train order
            keep = ~self._mask()
            pool = self.rand_order[keep[self.rand_order]].tolist()
            (self.rng if self.rng is not None else np.random).shuffle(pool)
            pick = np.asarray(pool[:q], np.int64)
            ops.mark_selected(self.excl, self.N, torch.from_numpy(pick).to(self.dev))
            self.n_selected += len(pick)
            return pick
        qs = self._slots()
        if self.mode == "mc":
            if committee is None:
                raise ValueError("mc mode needs `committee`")
            _, idx = self._mc(committee, layout, qs)
            ops.mark_selected(self.excl, self.N, idx)
        elif self.mode == "hc":
            _, idx = self._hc(qs)
            ops.mark_selected(self.excl, self.N, idx)
        else:  # mix: top-q of each part over the remaining songs, then the union's top-q
            if committee is None:
                raise ValueError("mix mode needs `committee`")
            vm, im = self._mc(committee, layout, qs)
            vh, ih = self._hc(qs, self.excl_hc)
            ih = torch.where(ih >= 0, ih + self.N, ih)
            _, idx = ops.topq_merge(torch.cat([vm, vh]), torch.cat([im, ih]), qs)
            # a song leaves both pools whichever part picked it (:484, :521-531)
            is_hc = idx >= self.N
            row = (idx - self.N).clamp(0, self.Nh - 1)
            item = idx.clamp(0, self.N - 1)
            song = torch.where(idx < 0, idx, torch.where(is_hc, self.h2m[row], idx))
            hrow = torch.where(idx < 0, idx, torch.where(is_hc, row, self.m2h[item]))
            ops.mark_selected(self.excl, self.N, song)
            ops.mark_selected(self.excl_hc, self.Nh, hrow)
        out = idx.cpu().numpy()
        out = out[out >= 0]
        if self.mode == "mix":
            # songs leaving the committee pool (an hc pick of a song outside it leaves only the table)
            self.n_selected += len(np.unique(song.cpu().numpy()[song.cpu().numpy() >= 0]))
        else:
            self.n_selected += len(out)
        return out

    def _mask(self):
        """The exclusion bitmap as a host bool array [N] (True = queried)."""
        words = self.excl.cpu().numpy().view(np.uint32)
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")
        return bits[: self.N].astype(bool)
