"""Host logic that needs no GPU: the groupby geometry, the C-ABI's argument
checks for the newer entry points, and the Python validation in front of them."""
import ctypes

import numpy as np
import pytest


def test_song_groups_matches_pandas_groupby():
    import pandas as pd

    from ce_amd import song_groups

    rng = np.random.default_rng(3)
    for grouped in (True, False):
        s_id = rng.integers(0, 50, 2000) * 3 + 11
        if grouped:
            s_id = np.sort(s_id)
        uniq, offsets, perm = song_groups(s_id)
        exp = pd.Series(np.arange(len(s_id)), index=s_id).groupby(level=0)
        assert np.array_equal(uniq, np.array(sorted(exp.groups)))
        assert (perm is None) == grouped
        order = np.arange(len(s_id)) if perm is None else perm
        for g, key in enumerate(uniq):
            rows = order[offsets[g]:offsets[g + 1]]
            assert np.array_equal(rows, np.flatnonzero(s_id == key))  # row order kept (stable)
    uniq, offsets, perm = song_groups(["b", "a", "b", "c"])
    assert list(uniq) == ["a", "b", "c"] and offsets.tolist() == [0, 1, 3, 4] and perm.tolist() == [1, 0, 2, 3]


def test_new_entry_points_validate_without_gpu():
    from ce_amd import _lib

    lib = _lib.load()
    p = ctypes.c_void_p(16)
    assert lib.ce_excl_words(0) == 0 and lib.ce_excl_words(33) == 2
    # a negative q is rejected; the two-stage API stops at CE_MAX_Q (ce_select_mc* take any q)
    rc = lib.ce_select_mc_excl(p, 0, 100, 4, 4, 16, 4, 1, p, -1, 0, p, 1 << 20, p, p, None)
    assert rc == _lib.CE_EINVAL
    rc = lib.ce_select_finish_cands(100, _lib.CE_MAX_Q + 1, p, 1 << 20, p, None)
    assert rc == _lib.CE_EUNSUPPORTED
    rc = lib.ce_select_mc_partial(p, 0, 100, 4, 4, 16, 4, 1, _lib.CE_MAX_Q + 1, 0, p, 1 << 20, None)
    assert rc == _lib.CE_EUNSUPPORTED
    rc = lib.ce_select_finish_cands(100, 10, p, 1 << 20, ctypes.c_void_p(24), None)  # misaligned records
    assert rc == _lib.CE_EINVAL
    rc = lib.ce_merge_cands(None, 8, 10, p, p, None)
    assert rc == _lib.CE_EINVAL
    # segment mean: bad dtype, bad strides
    rc = lib.ce_segment_mean(p, 2, 10, 4, 4, None, p, 3, p, 1, 4, None)
    assert rc == _lib.CE_EUNSUPPORTED
    rc = lib.ce_segment_mean(p, 1, 10, 4, 3, None, p, 3, p, 1, 4, None)
    assert rc == _lib.CE_EINVAL
    # member inference: too many features / classes, inconsistent K
    rc = lib.ce_gnb_predict_proba(p, 10, 513, 513, p, p, p, 4, p, 4, None)
    assert rc == _lib.CE_EINVAL
    for D in range(1, 8):  # fewer than 8 features: numpy's sequential sum, not the 8-lane plan
        assert lib.ce_gnb_predict_proba(p, 10, D, D, p, p, p, 4, p, 4, None) == _lib.CE_EUNSUPPORTED
    rc = lib.ce_sgd_predict_proba(p, 10, 260, 260, p, p, 3, 4, p, 4, None)
    assert rc == _lib.CE_EINVAL
    assert lib.ce_mark_selected(None, 10, p, 1, 0, None) == _lib.CE_EINVAL
    # one-launch records: q = 0 writes nothing (no launch), misaligned output rejected
    assert lib.ce_select_mc_cands(p, 0, 100, 4, 4, 16, 4, 1, 0, 0, p, 1 << 20, None, None) == _lib.CE_OK
    assert lib.ce_select_mc_cands(p, 0, 100, 4, 4, 16, 4, 1, 10, 0, p, 1 << 20, ctypes.c_void_p(24),
                                  None) == _lib.CE_EINVAL
    assert lib.ce_row_div_f64(p, p, -1, p, None) == _lib.CE_EINVAL


def test_frames_entry_validates_without_gpu():
    """ce_select_frames: member count, class count, dtype, q and workspace are
    checked on the host before anything launches."""
    from ce_amd import _lib
    from ce_amd.ops import _Member

    lib = _lib.load()
    p = ctypes.c_void_p(256)
    ws = lib.ce_select_frames_workspace_bytes(1000, 10)
    assert ws >= 65536 + 16 * 10
    mem = (_Member * 2)(_Member(256, 0, 0, 4), _Member(256, 1, 1, 4))
    args = lambda M, C, q, wsb, m=mem: (ctypes.cast(m, ctypes.c_void_p), M, C, p, None, 1000, q, 0, p, wsb, p, p,
                                        None)
    assert lib.ce_select_frames(*args(0, 4, 10, ws)) == _lib.CE_EINVAL          # no member
    assert lib.ce_select_frames(*args(33, 4, 10, ws)) == _lib.CE_EINVAL         # too many
    assert lib.ce_select_frames(*args(2, 5, 10, ws)) == _lib.CE_EUNSUPPORTED    # C = 5
    assert lib.ce_select_frames(*args(2, 4, -1, ws)) == _lib.CE_EINVAL          # q < 0
    assert lib.ce_select_frames(*args(2, 4, 65, ws)) == _lib.CE_EWORKSPACE      # q > 64: + the entropies
    assert lib.ce_select_frames_workspace_bytes(1000, 65) >= ws + 1000 * 8
    assert lib.ce_select_frames(*args(2, 4, 10, 64)) == _lib.CE_EWORKSPACE      # workspace
    bad = (_Member * 1)(_Member(256, 2, 0, 4))                                   # bf16 member
    assert lib.ce_select_frames(*args(1, 4, 10, ws, bad)) == _lib.CE_EUNSUPPORTED
    short = (_Member * 1)(_Member(256, 0, 0, 3))                                 # row stride < C
    assert lib.ce_select_frames(*args(1, 4, 10, ws, short)) == _lib.CE_EINVAL


def test_python_guards_without_gpu():
    torch = pytest.importorskip("torch")
    from ce_amd import ops

    with pytest.raises(ValueError, match="HIP device"):
        ops.segment_mean(torch.zeros((4, 4), dtype=torch.float64), torch.zeros(2, dtype=torch.int64))
    with pytest.raises(ValueError, match="HIP device"):
        ops.gnb_predict_proba(torch.zeros((4, 4), dtype=torch.float64), np.zeros((2, 4)), np.ones((2, 4)), [0.5, 0.5])
    with pytest.raises(ValueError, match="HIP device"):
        ops.merge_cands(torch.zeros((10, 2), dtype=torch.int64), 10)


def test_select_queries_guards_without_gpu():
    from ce_amd import select_queries
    from ce_amd.select import ConsensusEntropySelector

    with pytest.raises(ValueError, match="negative"):
        select_queries("mc", -1, committee=[np.zeros((3, 4))])
    assert select_queries("rand", 0, pool=[3, 1, 2]) == []
    with pytest.raises(ValueError, match="mode"):
        ConsensusEntropySelector(10, "qbc")
    sel = ConsensusEntropySelector(10, "mc")
    for empty in (None, [], np.zeros((0, 5, 4))):
        with pytest.raises(ValueError, match="pred_prob"):
            sel.select(pred_prob=empty)


def test_any_q_without_gpu():
    """Any q >= 0 (amg_test.py:547-553): q = 0 returns before any launch on every
    selecting entry point; q > CE_MAX_Q sizes the sort path's workspace (~40 B
    per item) and a too small workspace is still rejected on the host."""
    from ce_amd import _lib
    from ce_amd.ops import _Member

    lib = _lib.load()
    p = ctypes.c_void_p(256)
    big = _lib.CE_MAX_Q + 1
    N = 1_000_000
    assert lib.ce_select_mc(p, 0, N, 16, 4, 64, 4, 1, 0, 0, p, 1 << 20, None, None, None) == _lib.CE_OK
    assert lib.ce_select_mc_excl(p, 0, N, 16, 4, 64, 4, 1, p, 0, 0, p, 1 << 20, None, None, None) == _lib.CE_OK
    assert lib.ce_topq(p, N, 0, 0, p, 1 << 20, None, None, None) == _lib.CE_OK
    assert lib.ce_topq_merge(p, p, 4, 0, None, None, None) == _lib.CE_OK
    assert lib.ce_merge_cands(p, 4, 0, None, None, None) == _lib.CE_OK
    assert lib.ce_select_mix(p, 0, N, 4, 4, 4, 4 * N, 1, p, 100, 4, 0, p, 1 << 20, None, None, None) == _lib.CE_OK
    assert lib.ce_select_batched(p, 0, N, 4, 4, 4, 4 * N, 1, p, 10, 0, p, 1 << 20, None, None, None) == _lib.CE_OK
    assert lib.ce_select_mc_chunk(p, 0, N, 16, 4, 64, 4, 1, 0, 0, None, 1, p, 1 << 20, None) == _lib.CE_OK
    mem = (_Member * 1)(_Member(256, 0, 0, 4))
    assert lib.ce_select_frames(ctypes.cast(mem, ctypes.c_void_p), 1, 4, p, None, N, 0, 0, p, 1 << 20, None, None,
                                None) == _lib.CE_OK
    for f in (lambda q: lib.ce_select_mc_workspace_bytes(N, q), lambda q: lib.ce_topq_workspace_bytes(N, q),
              lambda q: lib.ce_select_mix_workspace_bytes(N, 1000, q),
              lambda q: lib.ce_select_batched_workspace_bytes(N, 500, q),
              lambda q: lib.ce_select_mc_chunk_workspace_bytes(N, q),
              lambda q: lib.ce_select_frames_workspace_bytes(N, q)):
        assert f(big) >= 40 * N > f(10)
    ws = lib.ce_select_mc_workspace_bytes(N, 10)  # big enough for the lists, not for the sort
    assert lib.ce_select_mc(p, 0, N, 16, 4, 64, 4, 1, big, 0, p, ws, p, p, None) == _lib.CE_EWORKSPACE
    assert lib.ce_select_mc(p, 0, N, 16, 4, 64, 4, 1, -5, 0, p, ws, p, p, None) == _lib.CE_EINVAL


def test_sort_path_rejects_2pow32_records_without_gpu():
    """The radix sort counts records in 32 bits (ce_launch_sort.hip): a pool of
    2^32 items or more with q > CE_MAX_Q is refused, not mis-sorted; batched
    users pack (user << 40 | position) and refuse 2^40 items."""
    from ce_amd import _lib

    lib = _lib.load()
    p = ctypes.c_void_p(256)
    q = _lib.CE_MAX_Q + 1
    big = 1 << 32
    huge_ws = (1 << 63) - 1
    rc = lib.ce_topq(p, big, q, 0, p, huge_ws, p, p, None)
    assert rc == _lib.CE_EUNSUPPORTED and b"2^32" in lib.ce_last_error()
    rc = lib.ce_select_mc(p, 0, big, 16, 4, 64, 4, 1, q, 0, p, huge_ws, p, p, None)
    assert rc == _lib.CE_EUNSUPPORTED
    rc = lib.ce_select_mc_cands(p, 0, big, 16, 4, 64, 4, 1, q, 0, p, huge_ws, p, None)
    assert rc == _lib.CE_EUNSUPPORTED
    rc = lib.ce_select_mix(p, 0, big - 5, 4, 4, 16, 4, 1, p, 10, 4, q, p, huge_ws, p, p, None)
    assert rc == _lib.CE_EUNSUPPORTED
    rc = lib.ce_select_batched(p, 0, 1 << 40, 4, 4, 16, 4, 1, p, 8, q, p, huge_ws, p, p, None)
    assert rc == _lib.CE_EUNSUPPORTED and b"2^40" in lib.ce_last_error()


def test_q_beyond_int32_is_rejected():
    """Every entry point takes q as int32: ops refuses a larger q instead of
    letting ctypes truncate it."""
    pytest.importorskip("torch")
    from ce_amd import ops

    assert ops._check_q(2**31 - 1) == 2**31 - 1
    with pytest.raises(ValueError, match="int32"):
        ops._check_q(2**32 + 3)
    with pytest.raises(ValueError, match="negative"):
        ops._check_q(-1)


def test_bench_traffic_only_for_the_launched_kernel(tmp_path, monkeypatch):
    """bench.py's roofline.traffic comes from profiles/traffic.json only when
    the record names the kernel this run launched (ce_last_kernel())."""
    import json

    import bench

    sym = "void ce::k_stream_nmc<0, 4, 16, 2, false>(ce::StreamArgs, int, ce::Cand*)"
    assert bench.kernel_symbol(sym) == "ce::k_stream_nmc<0, 4, 16, 2, false>"
    assert bench.kernel_symbol("ce::k<a<(1)>, 2>") == "ce::k<a<(1)>, 2>"
    path = tmp_path / "traffic.json"
    path.write_text(json.dumps({"NMC_k": {"kernel": sym, "hbm_bytes_per_launch": 123.0, "source": "x"}}))
    monkeypatch.setattr(bench, "TRAFFIC_FILE", str(path))
    assert bench.recorded_traffic("NMC_k", "ce::k_stream_nmc<0, 4, 16, 2, false>") == (123.0, "x")
    t, why = bench.recorded_traffic("NMC_k", "ce::k_stream_nmc<0, 4, 16, 2, true>")
    assert t is None and "this run launched" in why
    assert bench.recorded_traffic("NMC_k", "")[0] is None
    assert bench.recorded_traffic("MNC_k", "ce::k_stream_nmc<0, 4, 16, 2, false>")[0] is None


def test_committed_traffic_records_name_a_kernel():
    """Every committed traffic record names its exact kernel symbol and source profile."""
    import json
    import os

    from conftest import ROOT

    tr = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
    assert tr
    for key, e in tr.items():
        assert e["kernel"].startswith("void ce::k_") and "(" in e["kernel"], key
        assert e["hbm_bytes_per_launch"] > 0 and e["source"].startswith("profiles/"), key
        assert "k_stream_direct" not in e["kernel"], key


def test_bench_launch_plan():
    """bench.py --gpus N: one rank under torchrun (WORLD_SIZE set), N child
    ranks started by bench.py itself otherwise, and a refusal -- never a
    1-GPU line -- for a --gpus that WORLD_SIZE contradicts or that exceeds
    the visible GPUs outside a rehearsal."""
    import bench

    assert bench.launch_plan(1, {}, 0) == ("run", 1)  # N = 1 (the CPU box: the GPU call fails later, loudly)
    assert bench.launch_plan(1, {}, 8) == ("run", 1)
    assert bench.launch_plan(8, {}, 8) == ("spawn", 8)
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}, 8) == ("run", 8)
    assert bench.launch_plan(2, {"CE_AMD_REHEARSAL": "1"}, 1) == ("spawn", 2)
    assert bench.launch_plan(2, {"WORLD_SIZE": "2", "CE_AMD_REHEARSAL": "1"}, 1) == ("run", 2)
    for gpus, env, vis in ((8, {}, 1), (2, {"WORLD_SIZE": "1"}, 8), (1, {"WORLD_SIZE": "8"}, 8),
                           (8, {"WORLD_SIZE": "8"}, 4), (0, {}, 8)):
        with pytest.raises(SystemExit) as e:
            bench.launch_plan(gpus, env, vis)
        assert e.value.code == 2, (gpus, env, vis)
    env = bench.rank_env({"X": "1"}, 3, 8, 12345)
    assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"], env["MASTER_ADDR"], env["MASTER_PORT"], env["X"]) == \
        ("3", "3", "8", "127.0.0.1", "12345", "1")


def test_bench_refuses_without_gpus():
    """A plain `python3 bench.py --gpus 2` with no visible GPU exits 2 and
    prints no JSON line (here: the CPU container)."""
    import os
    import subprocess
    import sys

    from conftest import ROOT

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "CE_AMD_REHEARSAL")}
    env["HIP_VISIBLE_DEVICES"] = "-1" if env.get("HIP_VISIBLE_DEVICES") is None else env["HIP_VISIBLE_DEVICES"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 2 and r.stdout.strip() == "", (r.returncode, r.stdout, r.stderr[-500:])
    assert "visible GPU" in r.stderr


def test_bench_spawn_ranks_env_and_status(tmp_path):
    """bench.spawn_ranks starts N fresh processes with torchrun's variables
    (rank, world, one free 127.0.0.1 port) and returns the worst status: the
    failing rank's, 128 + signal for a killed one, 0 when all succeed."""
    import json
    import sys

    import bench

    child = tmp_path / "child.py"
    child.write_text(
        "import json, os, sys\n"
        "e = os.environ\n"
        f"open(os.path.join({str(tmp_path)!r}, 'r' + e['RANK']), 'w').write(json.dumps(\n"
        "    {k: e[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}))\n"
        "sys.exit(7 if e.get('FAIL_RANK') == e['RANK'] else 0)\n")
    code = str(child)
    assert bench.spawn_ranks([sys.executable, code], 3, poll_s=0.05) == 0
    seen = [json.loads((tmp_path / f"r{r}").read_text()) for r in range(3)]
    assert [s["RANK"] for s in seen] == ["0", "1", "2"] and {s["WORLD_SIZE"] for s in seen} == {"3"}
    assert {s["MASTER_ADDR"] for s in seen} == {"127.0.0.1"} and len({s["MASTER_PORT"] for s in seen}) == 1
    import os

    os.environ["FAIL_RANK"] = "1"
    try:
        assert bench.spawn_ranks([sys.executable, code], 3, poll_s=0.05) == 7
    finally:
        del os.environ["FAIL_RANK"]
    kill = "import os, signal; os.kill(os.getpid(), signal.SIGKILL) if os.environ['RANK'] == '0' else None"
    assert bench.spawn_ranks([sys.executable, "-c", kill], 2, poll_s=0.05) == 128 + 9
