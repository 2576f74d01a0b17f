"""Per-phase timing of the row coder inside the engine (diagnostic stamps).

Runs one warm-up batch and one measured batch of `--batch` frames with the
stamps on (cairo_ctx_set_debug(ctx, 2)) and prints, for the measured batch:
each frame's coding span inside the launch, the start lag between
consecutive frames, the mean duration of each phase of a macroblock, and the
producer-publish -> consumer-resume hand-off latency across rows.
usage: python tools/k2_phases.py [--config 720p] [--batch 8]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cairo_amd  # noqa: E402

CFG = {"720p": (1280, 720, 2, 16), "1080p": (1920, 1080, 4, 8), "4k": (3840, 2160, 4, 16), "cif": (352, 288, 4, 16)}
PHASES = ["wait", "window", "int_search", "subpel", "classify", "pred", "code", "publish", "window+drain"]

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="720p")
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--rows", type=int, default=0, help="row-coder workgroups (0 = default)")
ap.add_argument("--helpers", type=int, default=0, help="helper workgroups of the launch (0 = default: half)")
ap.add_argument("--row", type=int, default=10, help="MB row of the group timeline")
ap.add_argument("--frame", type=int, default=1, help="frame (>= 1) of the batch for the lag / group-timeline sections")
ap.add_argument("--db-chunk", type=int, default=64, help="deblock chunk width in luma columns (kernels.hip CAIRO_DB_CHUNK)")
ap.add_argument("--dump", default="", help="also save the raw stamps (npz) here")
a = ap.parse_args()
w, h, ring, q = CFG[a.config]
ctx = cairo_amd.Context(w, h, ring)
ctx.set_debug(2)
ctx.set_batch(a.batch)
if a.rows:
    ctx.set_workgroups(a.rows)
if a.helpers:
    ctx.set_helpers(a.helpers)
B = a.batch
for first in (0, B):  # warm-up batch, measured batch
    frames = [cairo_amd.make_band4(w, h, t) for t in range(first, first + B)]
    tks = [ctx.submit(f, first + i, first + i > 0, q) for i, f in enumerate(frames)]
    for t in tks:
        ctx.wait(t, copy=False)
        ctx.release(t)
st, dbs, kio, ist = ctx.read_stamps()  # 10 ns ticks
if a.dump:
    np.savez_compressed(a.dump, st=st[:B], dbs=dbs[:B], kio=kio, ist=ist[:B])
dbs = dbs[:B].astype(np.int64)
ist = ist[:B].astype(np.int64)
st = st[:B].astype(np.int64)
kio = kio.astype(np.int64)
hb, wb = st.shape[1:3]
steps = wb + 3 * (hb - 1)
t0 = kio[0]
print(f"{a.config} batch {B}: engine entry -> exit {(kio[1] - kio[0]) / 100.0:.1f} us "
      f"({(kio[1] - kio[0]) / 100.0 / B:.1f} us per frame)")
starts = []
for j in range(B):
    s0, s1 = st[j, ..., 0].min(), st[j, ..., 9].max()
    starts.append(s0)
    print(f"  frame {j}: coding {(s0 - t0) / 100.0:8.1f} .. {(s1 - t0) / 100.0:8.1f} us  "
          f"span {(s1 - s0) / 100.0:7.1f} us = {(s1 - s0) / 100.0 / steps:.2f} us/step")
if B > 1:
    lag = np.diff(np.array(starts)) / 100.0
    print(f"  start lag between frames: mean {lag.mean():.1f} us")
d = np.diff(st[..., :10], axis=-1) / 100.0  # (B, hmb, wmb, 9) us
print("per-MB phase means over the batch (us):")
for k, name in enumerate(PHASES):
    print(f"  {name:11s} mean {d[..., k].mean():8.3f}  p50 {np.median(d[..., k]):8.3f}")
tot = (st[..., 9] - st[..., 0]) / 100.0
print(f"  total/MB    mean {tot.mean():8.3f}")
lat = []
for j in range(B):
    for by in range(1, hb):
        for bx in range(wb):
            src = min(bx + 2, wb - 1)
            lat.append((st[j, by, bx, 1] - st[j, by - 1, src, 8]) / 100.0)  # pixel granules out at stamp 8
lat = np.array(lat)
print(f"  hand-off (publish -> resume) mean {lat.mean():.3f} p50 {np.median(lat):.3f} us")
clk = (st[..., 11] - st[..., 10]) / np.maximum(st[..., 9] - st[..., 0], 1) * 100.0  # MHz
print(f"  effective shader clock: mean {clk.mean():.0f} MHz")
# inter tasks: dequeue -> ready (dependency met) -> done
ok = ist[..., 2] > 0
if ok.any():
    wait = (ist[..., 1] - ist[..., 0])[ok] / 100.0
    run = (ist[..., 2] - ist[..., 1])[ok] / 100.0
    print(f"inter tasks: {ok.sum()}  wait mean {wait.mean():.1f} us  run mean {run.mean():.1f} us p50 {np.median(run):.1f} "
          f"max {run.max():.1f}")
    zm = (ist[..., 3] - ist[..., 1])[ok] / 100.0
    sw = ok & (ist[..., 4] > 0)
    l2 = ok & (ist[..., 7] > 0)
    print(f"  ready -> zero-MV checked mean {zm.mean():.1f} us; searched groups {sw.sum()} "
          f"({100.0 * sw.sum() / ok.sum():.0f} %): window staged after {((ist[..., 4] - ist[..., 3])[sw] / 100.0).mean():.1f} us, "
          f"staged -> done {((ist[..., 2] - ist[..., 4])[sw] / 100.0).mean():.1f} us (p50 "
          f"{np.median((ist[..., 2] - ist[..., 4])[sw] / 100.0):.1f})")
    if l2.any():
        l2r = ok & ((ist[..., 7] >> 16) > 0)
        print(f"  level-2 groups {l2.sum()} ({100.0 * l2.sum() / ok.sum():.1f} %; rows {l2r.sum()}, columns only "
              f"{(l2 & ~l2r).sum()}): wait+stage mean {((ist[..., 6] - ist[..., 5])[l2] / 100.0).mean():.1f} us; "
              f"their run mean {((ist[..., 2] - ist[..., 1])[l2] / 100.0).mean():.1f} us")
    nl2 = sw & ~l2
    if nl2.any():
        print(f"  level-1-only searched groups: staged -> done mean {((ist[..., 2] - ist[..., 4])[nl2] / 100.0).mean():.1f} us")
        seg = lambda a_, b_: ((ist[..., b_] - ist[..., a_])[nl2] / 100.0).mean()  # noqa: E731
        print(f"    staged -> step 16 done {seg(4, 8):.1f}, -> integer steps done {seg(8, 9):.1f}, -> sub-pel done "
              f"{seg(9, 10):.1f}, -> records released {seg(10, 2):.1f} us (first reference)")
    if wb <= 255:  # the row's helper deblock time (last per-row stamp slot)
        dbt = dbs[..., 255] / 100.0
        print(f"  helper deblock per row {dbt.mean():.1f} us = {dbt.mean() / max(1, ist.shape[2]):.1f} us per group")
    cu = ist[..., 11][ok]
    print(f"  after each group: deblock catch-up {np.mean(cu & 0xFFFFFFFF) / 100.0:.1f} us, "
          f"{np.mean(cu >> 32):.2f} chunks (of {(wb * 16 + a.db_chunk - 1) // a.db_chunk / max(1, ist.shape[2]):.2f} per group)")
    for j in range(B):
        okj = ist[j, ..., 2] > 0
        if okj.any() and j < 4:
            print(f"  frame {j}: inter tasks {(ist[j, ..., 0][okj].min() - t0) / 100.0:8.1f} .. "
                  f"{(ist[j, ..., 2][okj].max() - t0) / 100.0:8.1f} us")
# frame-to-frame lag of MB completion (stamp 9) at sample positions
F = min(max(a.frame, 1), B - 1)
if B > 2:
    js = [max(F - 1, 0), F, min(F + 1, B - 2)][: max(1, min(3, B - 1))]
    print(f"lag of frame j+1 behind frame j at MB (x, r), us [j={js}]:")
    for r in (0, 5, 10, 20, 30, 40, hb - 1):
        row = []
        for x in (0, wb // 2, wb - 1):
            lags = [(st[j + 1, r, x, 9] - st[j, r, x, 9]) / 100.0 for j in js]
            row.append(f"x={x:3d}: " + "/".join(f"{v:6.0f}" for v in lags))
        print(f"  r={r:3d}  " + "   ".join(row))
    # how long frame 1's MBs wait at group boundaries (wait phase at bx % 4 == 0)
    wt = (st[F, :, :, 1] - st[F, :, :, 0]) / 100.0
    print(f"frame {F} wait phase: at group starts mean {wt[:, 0::4].mean():.1f} us, elsewhere "
          f"{np.delete(wt, np.s_[0::4], axis=1).mean():.1f} us")
# deblock chunk k publish vs the coding of its last MB (stamp 9)
CH = a.db_chunk // 16
nch = (wb + CH - 1) // CH
for j in range(min(B, 2)):
    for r in (3, 10, 20, hb - 1):
        ks_ = [k for k in (1, nch // 4, nch // 2, nch - 2) if 0 <= k < nch]
        print(f"  frame {j} row {r}: deblock chunk k publish - its last MB coded, us: " + "  ".join(
            f"k={k}: {(dbs[j, r, k] - st[j, r, min(CH * k + CH - 1, wb - 1), 9]) / 100.0:.1f}" for k in ks_))
# frame 1, row 10: per group, when its inter task became ready / was claimed / done,
# and when the row coder reached / resumed at the group's first MB
if B > 1 and hb > 13 and (ist[..., 2] > 0).any():
    r = a.row if hasattr(a, 'row') else 10
    print(f"frame {F} row {r} per group (us): ready(deblock f{F - 1} row {r + 2}) wait-start ready done | coder reach resume")
    for g in range(0, (wb + 3) // 4, 3):
        need = min(64 * g + 80, w)  # level 1 of the inter window (kernels.hip inter_need_cols)
        kk = [k for k in range(min(nch, 255)) if (a.db_chunk * (k + 1) - 12 >= need or k == nch - 1)]
        ready = (dbs[F - 1, min(r + 2, hb - 1), kk[0]] - t0) / 100.0 if kk else float("nan")
        c, rd, dn = ((ist[F, r, g, k] - t0) / 100.0 for k in range(3))
        reach, res = (st[F, r, 4 * g, 0] - t0) / 100.0, (st[F, r, 4 * g, 1] - t0) / 100.0
        print(f"  g={g:2d}: {ready:8.1f} {c:8.1f} {rd:8.1f} {dn:8.1f} | {reach:8.1f} {res:8.1f}")
