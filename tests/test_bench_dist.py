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
