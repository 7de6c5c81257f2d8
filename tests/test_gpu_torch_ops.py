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


def _graph_nodes(g):
    """Node count of a kept (keep_graph=True) captured graph."""
    import ctypes

    import ce_amd

    f = ce_amd._lib.load().hipGraphGetNodes
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
    n = ctypes.c_size_t(0)
    assert f(ctypes.c_void_p(g.raw_cuda_graph()), None, ctypes.byref(n)) == 0
    return n.value


def test_graph_replays_1000_without_zero_fill(tops):
    """A captured select_mc (and select_batched / select_mix, sharing one
    carve on the capture stream) replayed 1000x equals the oracle on fresh
    pools: the workspace comes from the pre-zeroed graph arena (no zero-fill
    node in the graph, no fallback warning) and every replay leaves the
    arrival counters zero for the next."""
    import warnings

    import ce_amd.ops as ops
    from oracle import ce_oracle as O

    P = pool(71, (4, 1608, 4))
    Pb = pool(72, (4, 40 * 1608, 4))
    hc = torch.round(pool(73, (1608, 4)).double() * 1000) / 1000
    offs = torch.arange(0, 41, device="cuda", dtype=torch.int64) * 1608
    ops.select_mc(P, 10, "MNC")  # an eager call first: it creates the device's graph arena
    ops.reserve_graph_workspace(4 << 20)
    torch.cuda.synchronize()

    def capture():
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g):
            out = (ops.select_mc(P, 10, "MNC"), ops.select_batched(Pb, offs, 10, "MNC"),
                   ops.select_mix(P, hc, 10, "MNC"))
        g.instantiate()
        return g, out

    with warnings.catch_warnings():
        warnings.simplefilter("error")  # the fallback (a captured zero fill) warns
        g, ((v, i), (vb, ib), (vm, im)) = capture()
    carve = ops.WORKSPACE.arena.carve
    ops.WORKSPACE.arena.carve = lambda *a: None  # force the fallback: one zero fill per call
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            g_fill, _ = capture()
    finally:
        ops.WORKSPACE.arena.carve = carve
    n_arena, n_fill = _graph_nodes(g), _graph_nodes(g_fill)
    assert n_fill == n_arena + 3, (n_arena, n_fill)  # the arena's graph: the selection kernels only
    del g_fill
    for it in range(1000):
        if it % 250 == 0:
            P.copy_(pool(100 + it, P.shape))
            Pb.copy_(pool(200 + it, Pb.shape))
        g.replay()
        if it % 250 == 249 or it == 0:
            torch.cuda.synchronize()
            Pn = P.cpu().numpy().astype(np.float64)
            assert np.array_equal(i.cpu().numpy(), O.oracle_select_mc(Pn, 10)[1])
            assert np.array_equal(im.cpu().numpy(), O.oracle_select_mix(Pn, hc.cpu().numpy(), 10)[1])
            Pbn = Pb.cpu().numpy().astype(np.float64)
            for u in (0, 17, 39):
                eu = O.oracle_select_mc(np.ascontiguousarray(Pbn[:, u * 1608:(u + 1) * 1608]), 10)[1]
                assert np.array_equal(ib[u].cpu().numpy(), eu)
    torch.cuda.synchronize()


def test_dynamo_traces_one_node(tops):
    P = pool(4, (4, 5_000, 4))
    hc = pool(5, (5_000, 4)).double()

    def step(P, hc):
        v, i = torch.ops.ce_amd.select_mix(P, hc, 10, "MNC")
        return i + 0

    compiled = torch.compile(step, backend="eager", fullgraph=True)
    assert torch.equal(compiled(P, hc), step(P, hc))
    assert np.all(step(P, hc).cpu().numpy() >= 0)


def _oracle_idx(P, q):
    from oracle import ce_oracle as O

    return O.oracle_topq(O.oracle_committee_entropy(P.cpu().numpy(), "NMC"), q)[1]


def _idx(t):
    i = t.cpu().numpy()
    return i[i >= 0]


def test_two_streams_concurrently(tops):
    """ops.select_mc / select_batched issued back to back on two streams over
    different pools (the folded selection's arrival counters live in the
    workspace: one workspace per (device, stream), include/ce.h): every call on
    either stream equals the oracle."""
    import ce_amd.ops as ops

    Pa, Pb = pool(11, (1_000_000, 16, 4)), pool(12, (900_000, 16, 4))
    exp_a, exp_b = _oracle_idx(Pa, 10), _oracle_idx(Pb, 10)
    Ua = pool(13, (4, 500 * 1608, 4))
    offs = torch.arange(0, 500 * 1608 + 1, 1608, device="cuda", dtype=torch.int64)
    _, ub_ref = ops.select_batched(Ua, offs, 10, "MNC")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs_a, outs_b, outs_u = [], [], []
    for _ in range(12):
        with torch.cuda.stream(sa):
            outs_a.append(ops.select_mc(Pa, 10, "NMC")[1])
            outs_u.append(ops.select_batched(Ua, offs, 10, "MNC")[1])
        with torch.cuda.stream(sb):
            outs_b.append(ops.select_mc(Pb, 10, "NMC")[1])
    torch.cuda.synchronize()
    for i in outs_a:
        assert np.array_equal(_idx(i), exp_a)
    for i in outs_b:
        assert np.array_equal(_idx(i), exp_b)
    for i in outs_u:
        assert torch.equal(i, ub_ref)


def test_graph_replay_after_cache_growth(tops):
    """A captured selection keeps its own workspace: an eager call that grows
    the (device, stream) workspace cache after the capture does not free
    memory the graph uses, and the replay still equals the oracle."""
    import ce_amd.ops as ops

    P = pool(21, (200_000, 16, 4))
    ops.select_mc(P, 10, "NMC")  # an eager call first: the cache holds a small buffer
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        v, i = torch.ops.ce_amd.select_mc(P, 10, "NMC", 0)
    big = pool(22, (3_000_000, 16, 4))
    _, ib = ops.select_mc(big, 64, "NMC")  # grows the eager workspace (64-slot block lists)
    torch.cuda.synchronize()
    assert np.array_equal(_idx(ib), _oracle_idx(big, 64))
    P.copy_(pool(23, P.shape))
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(_idx(i), _oracle_idx(P, 10))


def test_workspace_cache_is_bounded(tops):
    """The (device, stream) workspace cache keeps at most MAX_STREAMS buffers
    (least recently used evicted): a caller cycling through short-lived streams
    does not pin one workspace per stream, and every call still equals the
    oracle; a sort-path call (q > CE_MAX_Q) gets a per-call workspace that the
    cache never holds."""
    import ce_amd.ops as ops

    P = pool(31, (300_000, 16, 4))
    exp = _oracle_idx(P, 10)
    torch.cuda.synchronize()
    n0 = len(ops.WORKSPACE)
    for _ in range(ops.WORKSPACE.MAX_STREAMS + 8):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            _, i = ops.select_mc(P, 10, "NMC")
        s.synchronize()
        assert np.array_equal(_idx(i), exp)
        assert len(ops.WORKSPACE) <= ops.WORKSPACE.MAX_STREAMS
    assert len(ops.WORKSPACE) == ops.WORKSPACE.MAX_STREAMS or n0 > ops.WORKSPACE.MAX_STREAMS
    key = (torch.cuda.current_device(), torch.cuda.current_stream().cuda_stream)
    before = ops.WORKSPACE._ws.get(key)
    nb = 0 if before is None else before.numel()
    q = 2049
    _, iq = ops.select_mc(P, q, "NMC")  # the sort path: ~40 B per item of per-call workspace
    torch.cuda.synchronize()
    after = ops.WORKSPACE._ws.get(key)
    assert (0 if after is None else after.numel()) == nb  # not cached
    assert np.array_equal(_idx(iq), _oracle_idx(P, q))


def test_last_kernel_names_the_stage1_kernel(tops):
    """ce_last_kernel() names the kernel a selection launched, in rocprofv3's
    form: bench.py ties its roofline.traffic record to it."""
    import ce_amd
    import ce_amd.ops as ops

    lib = ce_amd._lib.load()
    P = pool(41, (200_000, 16, 4))
    ops.select_mc(P, 10, "NMC")
    assert lib.ce_last_kernel().decode() == "ce::k_stream_nmc<0, 4, 16, 2, false, 2>"
    Pm = P.permute(1, 0, 2).contiguous()
    ops.select_mc(Pm, 10, "MNC")
    assert lib.ce_last_kernel().decode() == "ce::k_stream_nmc<0, 4, 16, 2, true, 2>"
    small = pool(42, (4, 1608, 4))
    ops.select_mc(small, 10, "MNC")
    assert lib.ce_last_kernel().decode().startswith("ce::k_select_tiles<ce::CommitteeSrc<0, 4, true>")
    ops.select_mc(P, 100, "NMC")  # q > 64: the block-synchronous lists, not a noted kernel
    assert lib.ce_last_kernel().decode() == ""
    # every selection entry point resets the name: a sort-path call after a noted one reports ""
    ops.select_mc(P, 10, "NMC")
    assert lib.ce_last_kernel().decode() != ""
    offs = torch.tensor([0, 100_000, 200_000], device="cuda", dtype=torch.int64)
    ops.select_batched(P.permute(1, 0, 2), offs, 3000, "MNC")
    assert lib.ce_last_kernel().decode() == ""
    ops.select_mc(P, 10, "NMC")
    ent = ops.committee_entropy(P, "NMC")
    ops.topq(ent, 3000)
    assert lib.ce_last_kernel().decode() == ""
    torch.cuda.synchronize()


def test_wide_chunks_grid_rule(tops):
    """The wide stream's grid (csrc/ce_launch_stream.hip): a launch with heavy
    items (>= 16 KiB) of >= 16384 items that folds its lists -- every chunk of
    a job, single selections -- runs the sampled floor + grid vote and launches
    BOTH grids (one block per CU with an 8-batch ring, and the occupancy grid;
    the one the vote does not pick exits at once: ce_last_kernel() names both);
    a smaller launch runs the occupancy grid alone -- and the job selects what
    one launch over the whole pool selects."""
    import ce_amd
    import ce_amd.ops as ops

    lib = ce_amd._lib.load()
    g = torch.Generator(device="cuda").manual_seed(55)
    P = torch.rand((50_000, 10, 1000), device="cuda", generator=g).to(torch.bfloat16)  # 20 KB items
    both = "ce::k_stream_wide2<2, 2, 2, 8>|ce::k_stream_wide2<2, 2, 2, 2>"
    job = ops.MCChunkJob(10, "NMC")
    job.add(P[:20_000])
    assert lib.ce_last_kernel().decode() == both
    job.add(P[20_000:40_000])
    assert lib.ce_last_kernel().decode() == both
    job.add(P[40_000:])
    assert lib.ce_last_kernel().decode() == "ce::k_stream_wide2<2, 2, 2, 2>"
    v, i = job.result()
    v1, i1 = ops.select_mc(P, 10, "NMC")
    assert lib.ce_last_kernel().decode() == both
    torch.cuda.synchronize()
    assert torch.equal(i, i1) and torch.equal(v.view(torch.int64), v1.view(torch.int64))