"""bench.py's multi-rank logic on CPU (gloo, world_size 2): the max-over-ranks
timing and the whole-job aggregate that rank 0 reports.  The GPU ranks run the
same functions over RCCL (bench.py main)."""
import os
import tempfile

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _worker(rank, world, store, out):
    # file rendezvous: no TCP port to race for
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    elapsed = 1.0 + rank  # rank 1 is the slow one
    m = bench.max_over_ranks(elapsed, dist, "cpu")
    out[rank] = (m, bench.aggregate_mpix(1280, 720, 10, world, m))
    dist.barrier()
    dist.destroy_process_group()


def test_max_over_ranks_and_aggregate_gloo():
    world = 2
    with tempfile.TemporaryDirectory() as tmp, mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(world, os.path.join(tmp, "store"), out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        m, v = res[r]
        assert m == pytest.approx(2.0)  # every rank sees the slowest rank's time
        assert v == pytest.approx(1280 * 720 * 10 * 2 / 2.0 / 1e6)


def _agree_worker(rank, world, store, out):
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    state = {"err": ""}
    ran = []

    def fail_on_rank1():
        ran.append("b")
        if rank == 1:
            raise RuntimeError("in-kernel wait timed out")

    oks = [bench.agreed_step(dist, None, rank, state, "a", lambda: ran.append("a")),
           bench.agreed_step(dist, None, rank, state, "b", fail_on_rank1),
           bench.agreed_step(dist, None, rank, state, "c", lambda: ran.append("c"))]
    dist.barrier()  # both ranks made the same collective calls: nothing is left waiting
    out[rank] = (oks, ran, state["err"])
    dist.destroy_process_group()


def test_agreed_step_stops_every_rank_gloo():
    """bench.py's single-stream leg: a failure on one rank stops every rank
    after the same step, with the same collective calls (no barrier left
    waiting for a rank that gave up)."""
    world = 2
    with tempfile.TemporaryDirectory() as tmp, mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_agree_worker, args=(world, os.path.join(tmp, "store"), out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        oks, ran, err = res[r]
        assert oks == [True, False, False]
        assert ran == ["a", "b"]  # step c ran nowhere
        assert ("in-kernel wait timed out" in err) if r == 1 else ("another rank failed" in err)


def test_single_rank_identity():
    assert bench.max_over_ranks(3.5, None, "cpu") == 3.5
    assert bench.aggregate_mpix(100, 100, 10, 1, 1.0) == pytest.approx(0.1)


def test_headline_field_selection():
    """The line's value (bench.headline): N = 1 the one context's stream; N > 1
    the single stream over all ranks (strong scaling, BASELINE.json
    configs[3]), with the replicas' aggregate only when that leg failed --
    labelled, never silently."""
    rep = {"value": 10000.0, "ms_per_step": 40.0}
    one = bench.headline(1, rep, None)
    assert (one["value"], one["scaling"], one["ms_per_step"]) == (10000.0, "weak", 40.0)
    single = {"value": 9000.0, "ms_per_step": 25.0}
    h = bench.headline(8, rep, single)
    assert (h["value"], h["scaling"], h["ms_per_step"]) == (9000.0, "strong", 25.0)
    assert "single_stream" in h["value_source"]
    bad = bench.headline(8, rep, {"error": ["rank 3 (timed): CairoError: ..."]})
    assert (bad["value"], bad["scaling"]) == (10000.0, "weak")
    assert "replicas" in bad["value_source"] and "rank 3" in bad["value_source"]
    assert bench.headline(2, rep, None)["value_source"].startswith("replicas")


def test_single_stream_check_covers_every_member():
    """>= 2N + R frames compared (each member twice, every mirror push), >= 8."""
    assert bench.single_stream_check_frames(8, 4, 84) == 20
    assert bench.single_stream_check_frames(2, 4, 84) == 8
    assert bench.single_stream_check_frames(4, 2, 84) == 10
    assert bench.single_stream_check_frames(8, 4, 12) == 12  # at most the warm-up frames


def _headline_worker(rank, world, store, out):
    """Every rank agrees on the single-stream result first (as bench.py's
    single_stream leg: all-reduced success and time), then selects."""
    import torch

    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    state = {"err": ""}

    def leg():
        if rank == 1:
            raise RuntimeError("in-kernel wait timed out: kind prev_progress")

    ok = bench.agreed_step(dist, None, rank, state, "timed", leg)
    el = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    errs = [None] * world
    dist.all_gather_object(errs, state["err"])
    single = {"value": 1.0 / float(el.item()), "ms_per_step": 1.0} if ok else {"error": [e for e in errs if e]}
    out[rank] = bench.headline(world, {"value": 3.0, "ms_per_step": 2.0}, single)
    dist.barrier()
    dist.destroy_process_group()


def test_headline_agrees_across_ranks_gloo():
    world = 2
    with tempfile.TemporaryDirectory() as tmp, mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_headline_worker, args=(world, os.path.join(tmp, "store"), out), nprocs=world, join=True)
        res = dict(out)
    assert res[0] == res[1]
    assert res[0]["scaling"] == "weak" and "rank 1" in res[0]["value_source"]
