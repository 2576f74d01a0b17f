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


def test_single_rank_identity():
    assert bench.max_over_ranks(3.5, None, "cpu") == 3.5
    assert bench.aggregate_mpix(100, 100, 10, 1, 1.0) == pytest.approx(0.1)
