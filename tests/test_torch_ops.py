"""The torch.library wrapper (ce_amd.torch_ops): the ops are registered under
torch.ops.ce_amd and their fake kernels give the output shapes without a
device (what dynamo / graph capture see).  GPU behaviour: test_gpu_torch_ops.py."""
import pytest

torch = pytest.importorskip("torch")


def test_ops_registered():
    import ce_amd.torch_ops  # noqa: F401

    for name in ("committee_entropy", "select_mc", "vote_table", "select_mix", "select_batched", "merge_cands"):
        assert hasattr(torch.ops.ce_amd, name), name


def test_fake_kernels_give_shapes():
    import ce_amd.torch_ops  # noqa: F401
    from torch._subclasses.fake_tensor import FakeTensorMode

    with FakeTensorMode():
        P = torch.empty((4, 1608, 4), dtype=torch.float32)
        ent = torch.ops.ce_amd.committee_entropy(P, "MNC")
        assert ent.shape == (1608,) and ent.dtype == torch.float64
        v, i = torch.ops.ce_amd.select_mc(P, 10, "MNC", 0)
        assert v.shape == (10,) and i.dtype == torch.int64
        v, i = torch.ops.ce_amd.select_batched(torch.empty((4, 5000, 4)), torch.empty(8, dtype=torch.int64), 10, "MNC")
        assert v.shape == (7, 10)
        f, e = torch.ops.ce_amd.vote_table(torch.empty((1608, 665), dtype=torch.int8), 4)
        assert f.shape == (1608, 4) and e.shape == (1608,)
        v, i = torch.ops.ce_amd.select_mix(P, torch.empty((1608, 4), dtype=torch.float64), 10, "MNC")
        assert i.shape == (10,)
        with pytest.raises(ValueError):
            torch.ops.ce_amd.select_mc(P, 10, "XYZ", 0)
