"""Per-phase timing of the macroblock wavefront kernel (k_mb_rows).

Runs a few frames with the diagnostic stamps on (cairo_ctx_set_debug(ctx, 2))
and prints the mean duration of each phase of a macroblock, plus the
producer-publish -> consumer-resume hand-off latency across rows.
usage: python tools/k2_phases.py [--config 720p] [--frames 4]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cairo_amd  # noqa: E402

CFG = {"720p": (1280, 720, 2, 16), "1080p": (1920, 1080, 4, 8), "4k": (3840, 2160, 4, 16), "cif": (352, 288, 4, 16)}
PHASES = ["wait", "window", "int_search", "subpel", "classify", "pred", "code", "store", "publish"]

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="720p")
ap.add_argument("--frames", type=int, default=4)
a = ap.parse_args()
w, h, ring, q = CFG[a.config]
ctx = cairo_amd.Context(w, h, ring)
ctx.set_debug(2)
for t in range(a.frames):
    ctx.encode_frame(cairo_amd.make_band4(w, h, t), t, t > 0, q)
    ctx.sync()
st, dbs, kio = ctx.read_stamps()  # 10 ns ticks
kio = kio.astype(np.int64)
st, dbs = st.astype(np.int64), dbs.astype(np.int64)
d = np.diff(st[..., :10], axis=2) / 100.0  # us
print(f"{a.config} frame {a.frames - 1}: per-MB phase means (us) over {st.shape[0] * st.shape[1]} MBs")
for k, name in enumerate(PHASES):
    print(f"  {name:11s} mean {d[..., k].mean():8.3f}  p50 {np.median(d[..., k]):8.3f}  max {d[..., k].max():8.3f}")
tot = (st[..., 9] - st[..., 0]) / 100.0
print(f"  total/MB    mean {tot.mean():8.3f}")
# hand-off: MB (bx, by) resumes (stamp 1) after (bx+2, by-1) published (stamp 9)
hb, wb = st.shape[:2]
lat = []
for by in range(1, hb):
    for bx in range(wb):
        src = min(bx + 2, wb - 1)
        lat.append((st[by, bx, 1] - st[by - 1, src, 9]) / 100.0)
lat = np.array(lat)
print(f"  hand-off (publish -> resume) mean {lat.mean():.3f} p50 {np.median(lat):.3f} us")
clk = (st[..., 11] - st[..., 10]) / np.maximum(st[..., 9] - st[..., 0], 1) * 100.0  # MHz
print(f"  effective shader clock: mean {clk.mean():.0f} MHz, p10 {np.percentile(clk, 10):.0f}, p90 {np.percentile(clk, 90):.0f}")
span = (st[..., 9].max() - st[..., 0].min()) / 100.0
print(f"  kernel span {span:.1f} us, steps {wb + 3 * (hb - 1)}, per step {span / (wb + 3 * (hb - 1)):.3f} us")
# deblock workers: per row, phases relative to the row-coded publish (stamp 8)
DBP = ["wait", "acquire", "table", "H band0", "V band0", "H band1", "V band1+pub"]
dd = np.diff(dbs[:, :8], axis=1) / 100.0
print("deblock per row (us): " + ", ".join(f"{n} {dd[:, k].mean():.2f}" for k, n in enumerate(DBP)))
lag = (dbs[:, 7] - dbs[:, 8]) / 100.0
print(f"  row coded -> row deblocked: mean {lag.mean():.2f} us, last row {lag[-1]:.2f} us")
print(f"  last MB end -> last row deblocked: {(dbs[:, 7].max() - st[..., 9].max()) / 100.0:.2f} us")
print(f"  kernel entry -> first MB: {(st[..., 0].min() - kio[0]) / 100.0:.2f} us; "
      f"last row deblocked -> kernel exit: {(kio[1] - dbs[:, 7].max()) / 100.0:.2f} us; "
      f"entry -> exit {(kio[1] - kio[0]) / 100.0:.1f} us")
