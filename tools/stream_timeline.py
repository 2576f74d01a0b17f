"""Timeline of the frame pipeline (cairo_stream_*): where a frame's time goes
between submit and collect, and the steady-state period of each stage.
usage: python tools/stream_timeline.py [--config 720p] [--frames 160] [--threads 14] [--batch 16]"""
import argparse
import os
import sys
from collections import deque

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cairo_amd  # noqa: E402

CFG = {"720p": (1280, 720, 2, 16), "1080p": (1920, 1080, 4, 8), "4k": (3840, 2160, 4, 16)}
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="720p")
ap.add_argument("--frames", type=int, default=160)
ap.add_argument("--threads", type=int, default=14)
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--distinct", action="store_true", help="every frame distinct content (as bench.py), else 8 cycled")
ap.add_argument("--ctx-only", action="store_true", help="hot path alone through cairo_ctx_* (no stream), total time only")
a = ap.parse_args()
w, h, ring, q = CFG[a.config]
import torch  # device-resident inputs, as in bench.py

dev = torch.device("cuda:0")
nsrc = a.frames if a.distinct else 8
frames = [torch.from_numpy(cairo_amd.make_band4(w, h, t)).to(dev) for t in range(nsrc)]
ctx = cairo_amd.Context(w, h, ring)
ctx.set_batch(a.batch)
if a.ctx_only:
    import time

    stages = ctx.L.cairo_ctx_stages(ctx.h)
    inflight = deque()
    t0 = time.perf_counter()
    for f in range(a.frames):
        if len(inflight) == stages:
            tk = inflight.popleft()
            ctx.wait(tk, copy=False)
            ctx.release(tk)
        inflight.append(ctx.submit(frames[f % nsrc].data_ptr(), f, f > 0, q, on_device=True))
    while inflight:
        tk = inflight.popleft()
        ctx.wait(tk, copy=False)
        ctx.release(tk)
    print(f"ctx only: total {(time.perf_counter() - t0) * 1e3:.1f} ms for {a.frames} frames")
    sys.exit(0)
st = cairo_amd.Stream(ctx, threads=a.threads)
stages = ctx.L.cairo_ctx_stages(ctx.h)
out = np.zeros(w * h * 4, np.uint8)
inflight, tl = deque(), []
for f in range(a.frames):
    if len(inflight) == stages:
        tk = inflight.popleft()
        st.collect(tk, out, 0)
        tl.append(st.timeline(tk))
    inflight.append(st.submit(frames[f % nsrc].data_ptr(), f, f > 0, q, on_device=True))
while inflight:
    tk = inflight.popleft()
    st.collect(tk, out, 0)
    tl.append(st.timeline(tk))
st.close()
T = np.array(tl)
print(f"total {(T[-1, 4] - T[0, 0]) / 1e3:.1f} ms for {a.frames} frames")
T = T[a.frames // 4:]  # steady state
names = ["submit->outputs", "outputs->entropy start", "entropy", "entropy end->collect"]
for k, n in enumerate(names):
    d = (T[:, k + 1] - T[:, k]) / 1e3
    print(f"{n:24s} mean {d.mean():7.2f} ms  p50 {np.median(d):7.2f}  max {d.max():7.2f}")
for k, n in enumerate(["submit", "outputs", "entropy start", "entropy end", "collect"]):
    print(f"period of {n:14s} {np.diff(T[:, k]).mean() / 1e3:.3f} ms/frame")
