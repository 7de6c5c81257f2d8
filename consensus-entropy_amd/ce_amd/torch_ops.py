"""torch.library custom operators over the C-ABI ("a
thin torch.library custom-op wrapper"; north star: "a thin PyTorch-ROCm
custom-op / C-ABI layer").  Importing this module registers, in the
``ce_amd`` namespace:

  torch.ops.ce_amd.committee_entropy(P, layout) -> ent [N] f64           amg_test.py:441-443
  torch.ops.ce_amd.select_mc(P, q, layout, base_idx) -> (vals, idx)       :441-445
  torch.ops.ce_amd.vote_table(votes, C) -> (freq [N, C], ent [N])        :109-117
  torch.ops.ce_amd.select_mix(P, hc, q, layout) -> (vals, idx)            :473-480
  torch.ops.ce_amd.select_batched(P, offsets, q, layout) -> (vals, idx)   :345 loop
  torch.ops.ce_amd.merge_cands(cands, q) -> (vals, idx)                   multi-GPU merge

Each op runs the same HIP kernels as ce_amd.ops (device tensors only, on the
current stream, no host synchronisation), and has a fake (meta) kernel giving
its output shapes, so the ops are visible to torch.ops, dynamo tracing
(torch.compile) and HIP-graph capture.  The kernels' outputs are fresh tensors:
nothing is mutated.
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import ops

_LIB = "ce_amd"


def _n_items(P: torch.Tensor, layout: str) -> int:
    if layout not in ("MNC", "NMC"):
        raise ValueError(f"layout must be 'MNC' or 'NMC', got {layout!r}")
    return P.shape[1] if layout == "MNC" else P.shape[0]


def _sel_fake(dev, lead, q):
    return (torch.empty((*lead, q), dtype=torch.float64, device=dev),
            torch.empty((*lead, q), dtype=torch.int64, device=dev))


@torch.library.custom_op(f"{_LIB}::committee_entropy", mutates_args=())
def committee_entropy(P: torch.Tensor, layout: str) -> torch.Tensor:
    return ops.committee_entropy(P, layout)


@committee_entropy.register_fake
def _(P, layout):
    return torch.empty((_n_items(P, layout),), dtype=torch.float64, device=P.device)


@torch.library.custom_op(f"{_LIB}::select_mc", mutates_args=())
def select_mc(P: torch.Tensor, q: int, layout: str, base_idx: int) -> Tuple[torch.Tensor, torch.Tensor]:
    return ops.select_mc(P, q, layout, base_idx)


@select_mc.register_fake
def _(P, q, layout, base_idx):
    _n_items(P, layout)
    return _sel_fake(P.device, (), q)


@torch.library.custom_op(f"{_LIB}::vote_table", mutates_args=())
def vote_table(votes: torch.Tensor, C: int) -> Tuple[torch.Tensor, torch.Tensor]:
    return ops.vote_table(votes, C)


@vote_table.register_fake
def _(votes, C):
    N = votes.shape[0]
    return (torch.empty((N, C), dtype=torch.float64, device=votes.device),
            torch.empty((N,), dtype=torch.float64, device=votes.device))


@torch.library.custom_op(f"{_LIB}::select_mix", mutates_args=())
def select_mix(P: torch.Tensor, hc: torch.Tensor, q: int, layout: str) -> Tuple[torch.Tensor, torch.Tensor]:
    return ops.select_mix(P, hc, q, layout)


@select_mix.register_fake
def _(P, hc, q, layout):
    _n_items(P, layout)
    return _sel_fake(P.device, (), q)


@torch.library.custom_op(f"{_LIB}::select_batched", mutates_args=())
def select_batched(P: torch.Tensor, offsets: torch.Tensor, q: int, layout: str) -> Tuple[torch.Tensor, torch.Tensor]:
    return ops.select_batched(P, offsets, q, layout)


@select_batched.register_fake
def _(P, offsets, q, layout):
    return _sel_fake(P.device, (offsets.shape[0] - 1,), q)


@torch.library.custom_op(f"{_LIB}::merge_cands", mutates_args=())
def merge_cands(cands: torch.Tensor, q: int) -> Tuple[torch.Tensor, torch.Tensor]:
    return ops.merge_cands(cands, q)


@merge_cands.register_fake
def _(cands, q):
    return _sel_fake(cands.device, (), q)
