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
        cairo.task_order(10, 33)
