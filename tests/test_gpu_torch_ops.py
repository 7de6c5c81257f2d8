"""torch.ops.ce_amd on the GPU: same answers as ce_amd.ops, captured in a HIP
graph, and traced by dynamo (torch.compile, eager backend: no generated
kernels) as single graph nodes."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tops():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ce_amd
    import ce_amd.ops  # noqa: F401
    import ce_amd.torch_ops as T

    ce_amd.load()
    return T


def pool(seed, shape):
    g = torch.Generator(device="cuda").manual_seed(seed)
    e = -torch.log(torch.rand(shape, device="cuda", generator=g).clamp_min_(1e-30))
    return e / e.sum(-1, keepdim=True)


def test_ops_equal_direct_calls(tops):
    import ce_amd.ops as ops

    P = pool(1, (4, 20_000, 4))
    assert torch.equal(torch.ops.ce_amd.committee_entropy(P, "MNC"), ops.committee_entropy(P, "MNC"))
    v, i = torch.ops.ce_amd.select_mc(P, 10, "MNC", 0)
    v2, i2 = ops.select_mc(P, 10, "MNC")
    assert torch.equal(i, i2) and torch.equal(v, v2)
    offs = torch.arange(0, 20_001, 1000, device="cuda", dtype=torch.int64)
    _, ib = torch.ops.ce_amd.select_batched(P, offs, 10, "MNC")
    assert torch.equal(ib, ops.select_batched(P, offs, 10, "MNC")[1])


def test_hip_graph_capture(tops):
    P = pool(2, (200_000, 16, 4))
    torch.ops.ce_amd.select_mc(P, 10, "NMC", 0)  # warm the workspace cache outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        v, i = torch.ops.ce_amd.select_mc(P, 10, "NMC", 0)
    P.copy_(pool(3, P.shape))
    g.replay()
    torch.cuda.synchronize()
    _, ie = torch.ops.ce_amd.select_mc(P, 10, "NMC", 0)
    assert torch.equal(i, ie)


def test_dynamo_traces_one_node(tops):
    P = pool(4, (4, 5_000, 4))
    hc = pool(5, (5_000, 4)).double()

    def step(P, hc):
        v, i = torch.ops.ce_amd.select_mix(P, hc, 10, "MNC")
        return i + 0

    compiled = torch.compile(step, backend="eager", fullgraph=True)
    assert torch.equal(compiled(P, hc), step(P, hc))
    assert np.all(step(P, hc).cpu().numpy() >= 0)
