"""Frame-interleaved groups on the CPU: the partition and ownership logic
(cairo_amd.group_layout mirrors backend.hip frame_links) and the exchange of
member records between processes (gloo, world_size 2), as bench.py's
single-stream leg does it over the ranks of a node."""
import os
import tempfile

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import cairo_amd


@pytest.mark.parametrize("size", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("ring", [2, 3, 4])
def test_layout_invariants(size, ring):
    stages = 8
    frames = 200
    lay = [cairo_amd.group_layout(n, size, ring, stages) for n in range(frames)]
    # partition: member n % N, tickets consecutive per member
    for k in range(size):
        mine = [n for n in range(frames) if lay[n]["member"] == k]
        assert [lay[n]["ticket"] for n in mine] == list(range(len(mine)))
    # a reconstruction slot is next written by a frame >= R later (its last
    # reader is frame n + R: the stale rows); == R exactly when in place
    holder = {}
    for n in range(frames):
        key = (lay[n]["member"], lay[n]["recon_slot"])
        if key in holder:
            gap = n - holder[key]
            assert gap >= ring
            assert (gap == ring) == lay[n]["in_place"]
        holder[key] = n
    if size == 1:
        assert all(x["in_place"] for x in lay) and lay[0]["recon_slots"] == ring
    # a staging slot (output_cache, progress words) is reused N * stages frames later
    seen = {}
    for n in range(frames):
        key = (lay[n]["member"], lay[n]["staging_slot"])
        if key in seen:
            assert n - seen[key] == size * stages
        seen[key] = n


@pytest.mark.parametrize("size", [2, 3, 4, 5, 8, 16])
@pytest.mark.parametrize("ring", [2, 3, 4])
def test_mirror_layout(size, ring):
    """Members on other devices / processes keep every frame they read in a
    local mirror slot (backend.hip frame_links, mirror mode): the slots fit
    the ring every member allocates, a slot is rewritten only by the same
    producer's frame N * S >= R later, and each frame is pushed to exactly the
    other members holding its R-1 referencing frames and its stale-row reader."""
    frames = 200
    lay = [cairo_amd.group_layout(n, size, ring, 8, mirror=True) for n in range(frames)]
    S = -(-ring // size)
    assert size * S <= cairo_amd.MIRROR_SLOTS
    holder = {}
    for n in range(frames):
        slot = lay[n]["recon_slot"]
        assert slot // S == n % size  # the producer's block
        if slot in holder:
            assert n - holder[slot] == size * S >= ring
        holder[slot] = n
        want = {(n + d) % size for d in range(1, ring + 1)} - {n % size}
        assert set(lay[n]["readers"]) == want and len(lay[n]["readers"]) <= 4
        # every frame n reads (n-1..n-R) is local: produced here or pushed here
        for d in range(1, ring + 1):
            if n - d >= 0:
                src = lay[n - d]
                assert src["member"] == n % size or n % size in src["readers"]


def _rank(rank, world, store, out):
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    rec = bytes([rank]) * cairo_amd.PEER_SIZE  # stands in for Context.peer_info()
    recs = [None] * world
    dist.all_gather_object(recs, rec)
    frames = [n for n in range(40) if cairo_amd.group_layout(n, world, 4, 64)["member"] == rank]
    out[rank] = ([r[0] for r in recs], frames)
    dist.barrier()
    dist.destroy_process_group()


def test_record_exchange_and_partition_gloo():
    world = 2
    with tempfile.TemporaryDirectory() as tmp, mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_rank, args=(world, os.path.join(tmp, "store"), out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        assert res[r][0] == list(range(world))  # every rank holds all records, in rank order
    a, b = res[0][1], res[1][1]
    assert sorted(a + b) == list(range(40)) and not set(a) & set(b)
