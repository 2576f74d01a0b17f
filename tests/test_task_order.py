"""The engine's task order and the shared-pool merge (CPU, no device).

k_engine's workers dequeue (frame, row) tasks in the launch's task order
(`cairo_task_order`, backend.hip task_order) and, with the pools shared, also
the previous launch's remaining tasks, taking whichever queue's next task has
the smaller key row + slope * frame (the previous launch's frames first;
kernels.hip next_task).  Deadlock freedom needs every task's
waits to point to tasks earlier in that merged order: a row waits for the row
above in its frame (granules, deblock progress) and for rows r+2 / r+3 of the
previous frame (the helpers' window levels, encode.cpp's serial order:
SURVEY.md A9, A20).
"""
import itertools

import numpy as np
import pytest

import cairo_amd


def _merge(prev, cur, slope):
    """next_task's choice between two queues, replayed sequentially."""
    pframes = (max(int(o) >> 16 for o in prev) + 1) if len(prev) else 0
    out, i, j = [], 0, 0
    while i < len(prev) or j < len(cur):
        if i < len(prev) and j < len(cur):
            op, ob = int(prev[i]), int(cur[j])
            usep = (op & 0xFFFF) + slope * (op >> 16) <= (ob & 0xFFFF) + slope * (pframes + (ob >> 16))
        else:
            usep = i < len(prev)
        if usep:
            out.append((int(prev[i]) >> 16, int(prev[i]) & 0xFFFF))
            i += 1
        else:
            out.append((pframes + (int(cur[j]) >> 16), int(cur[j]) & 0xFFFF))
            j += 1
    return out


def _deps(f, r, hmb):
    d = []
    if r > 0:
        d.append((f, r - 1))
    if f > 0:
        d.append((f - 1, min(r + 3, hmb - 1)))
    return d


@pytest.mark.parametrize("hmb", [1, 3, 18, 45, 68, 135])
def test_launch_order_is_a_sorted_permutation(cairo, hmb):
    for frames in (1, 2, 7, 24, 32):
        o, slope = cairo.task_order(hmb, frames)
        tasks = [(int(x) >> 16, int(x) & 0xFFFF) for x in o]
        assert sorted(tasks) == [(f, r) for f in range(frames) for r in range(hmb)]
        keys = [r + slope * f for f, r in tasks]
        assert keys == sorted(keys)


@pytest.mark.parametrize("hmb", [1, 3, 18, 68, 135])
def test_merged_order_respects_every_wait(cairo, hmb):
    """Two consecutive launches of any sizes: in the merged order every task
    comes after every task it waits for."""
    for n1, n2 in itertools.product((1, 2, 5, 24, 32), (1, 3, 24, 32)):
        p, slope = cairo.task_order(hmb, n1)
        c, _ = cairo.task_order(hmb, n2)
        merged = _merge(p, c, slope)
        assert sorted(merged) == [(f, r) for f in range(n1 + n2) for r in range(hmb)]
        pos = {t: k for k, t in enumerate(merged)}
        for (f, r), k in pos.items():
            for d in _deps(f, r, hmb):
                assert pos[d] < k, (hmb, n1, n2, (f, r), d)


def test_merged_order_interleaves_the_tail(cairo):
    """The merge is not "previous launch first": the next launch's first rows
    come before the previous launch's last frame's bottom rows (the tail whose
    waits are long), which is what lets both launches share their workers."""
    hmb = 135
    p, slope = cairo.task_order(hmb, 24)
    c, _ = cairo.task_order(hmb, 24)
    merged = _merge(p, c, slope)
    first_new = next(k for k, (f, _) in enumerate(merged) if f >= 24)
    last_old = max(k for k, (f, _) in enumerate(merged) if f < 24)
    assert first_new < last_old


def test_task_order_rejects_bad_sizes(cairo):
    with pytest.raises(cairo.CairoError):
        cairo.task_order(0, 1)
    with pytest.raises(cairo.CairoError):
        cairo.task_order(10, 49)


@pytest.mark.parametrize("hmb", [3, 18, 45, 68, 99, 100, 135, 270])
def test_label_queues_partition_the_order(cairo, hmb):
    """XCD-banded queues (kernels.h kLabels): each label's queue is the
    launch's task order restricted to that label's rows, a contiguous band."""
    for frames in (1, 2, 7, 28, 32, 40, 48):
        o, slope = cairo.task_order(hmb, frames)
        q, seg, nlab = cairo.task_queues(hmb, frames)
        assert nlab == (8 if hmb >= 100 else 1)
        # the launch's own predicate: both worker counts split over the 8 labels
        assert cairo.task_queues(hmb, frames, helpers=191, rows=193)[2] == 1
        assert cairo.task_queues(hmb, frames, helpers=96, rows=96, pool=1)[2] == nlab
        assert seg[0] == 0 and list(seg) == sorted(seg) and seg[nlab] == frames * hmb
        assert all(seg[l] == frames * hmb for l in range(nlab, 9))
        lab_of = lambda x: (int(x) & 0xFFFF) * 8 // hmb if nlab == 8 else 0
        for lab in range(nlab):
            mine = list(q[seg[lab]:seg[lab + 1]])
            assert mine == [x for x in o if lab_of(x) == lab]
        if nlab == 8:  # contiguous bands, every label has rows
            bands = [sorted({int(x) & 0xFFFF for x in q[seg[l]:seg[l + 1]]}) for l in range(8)]
            assert all(b and b == list(range(b[0], b[-1] + 1)) for b in bands)


def _simulate(queues, workers, deps, key, steal=None):
    """Per-label worker pools taking their label's queue in order (with
    steal = W: another label's head instead when it is more than W keys
    earlier, or when the own queue is exhausted: kernels.hip next_task); a
    task finishes once everything it waits for has finished.  -> finished
    count."""
    done, heads = set(), [0] * len(queues)
    held = [[None] * workers for _ in queues]
    total = sum(len(q) for q in queues)
    inf = float("inf")

    def take(lab):
        ks = [key(q[heads[l]]) if heads[l] < len(q) else inf for l, q in enumerate(queues)]
        if min(ks) == inf:
            return None
        z = lab
        if steal is not None and (ks[lab] == inf or ks[lab] - min(ks) > steal):
            z = ks.index(min(ks))
        if ks[z] == inf:
            return None
        heads[z] += 1
        return queues[z][heads[z] - 1]

    while len(done) < total:
        moved = False
        for lab in range(len(queues)):
            for w in range(workers):
                t = held[lab][w]
                if t is None:
                    t = held[lab][w] = take(lab)
                    moved |= t is not None
                if t is not None and all(d in done for d in deps(t)):
                    done.add(t)
                    held[lab][w] = None
                    moved = True
        if not moved:
            break
    return len(done)


@pytest.mark.parametrize("hmb", [100, 135])
@pytest.mark.parametrize("steal", [None, 0, 2, 7])
def test_label_queues_cannot_deadlock(cairo, hmb, steal):
    """Two consecutive launches, every label merging the previous launch's
    queue with its own (next_task), with or without stealing: with a single
    worker per label every task still finishes, whatever the label of the
    rows it waits for."""
    n1, n2 = 5, 3
    p, seg1, _ = cairo.task_queues(hmb, n1)
    c, seg2, _ = cairo.task_queues(hmb, n2)
    _, slope = cairo.task_order(hmb, 1)
    queues = []
    for lab in range(8):
        # every label has rows of every frame, so _merge numbers the second
        # launch's frames from n1, as next_task does (ptotal / hmb)
        queues.append(_merge(p[seg1[lab]:seg1[lab + 1]], c[seg2[lab]:seg2[lab + 1]], slope))
    n = _simulate(queues, 1, lambda t: _deps(t[0], t[1], hmb), lambda t: t[1] + slope * t[0], steal)
    assert n == (n1 + n2) * hmb
