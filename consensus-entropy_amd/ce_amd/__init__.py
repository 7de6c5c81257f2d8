"""ce_amd -- MI355X-native consensus-entropy query selection.

Drop-in for the selection path of juansgomez87/consensus-entropy
(amg_test.py:425-489): committee consensus entropy (mc), human-consensus vote
entropy (hc), their row-stacked union (mix) and the random baseline (rand),
computed by hand-written gfx950 HIP kernels behind the C-ABI of include/ce.h.
"""
from ._lib import CE_MAX_Q, CEError, load  # noqa: F401
from .select import (MODES, ConsensusEntropySelector, committee_from_frames, select_from_frames, select_queries,  # noqa: F401
                     song_groups, stack_committee)

from .session import SelectionSession  # noqa: F401,E402

__all__ = ["SelectionSession", "select_queries", "ConsensusEntropySelector", "stack_committee", "committee_from_frames",
           "select_from_frames", "song_groups",
           "MODES", "CE_MAX_Q", "CEError", "load", "ops", "dist", "torch_ops"]


def __getattr__(name):  # lazy submodules (ops/dist need torch)
    if name in ("ops", "dist", "torch_ops"):
        import importlib

        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
