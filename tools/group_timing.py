"""Throughput of one stream encoded by a frame-interleaved group of N member
contexts in this process, against one context, on the GPUs
given (default: N members on device 0, each with 1/N of the workgroup slots).
Frames resident in HBM, band4, timed like bench.py (Mpix/s).  Needs
GPU_MAX_HW_QUEUES >= 3 N + 2 in the environment.
usage: python tools/group_timing.py [--config 4k] [--members 2] [--frames 160] [--devices 0,0]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4k", choices=sorted(bench.CONFIGS))
    ap.add_argument("--members", type=int, default=2)
    ap.add_argument("--frames", type=int, default=160)
    ap.add_argument("--devices", default="")
    a = ap.parse_args()
    import torch

    import cairo_amd

    w, h, ring, q, _ = bench.CONFIGS[a.config]
    devs = [int(x) for x in a.devices.split(",")] if a.devices else [0] * a.members
    n = a.frames + 32
    frames = {}
    for d in sorted(set(devs)):
        frames[d] = torch.empty((n, h, w, 3), dtype=torch.uint8, device=torch.device("cuda", d))
        for f in range(n):
            frames[d][f].copy_(torch.from_numpy(cairo_amd.make_band4(w, h, f)))
    torch.cuda.synchronize()

    def ptr(d, f):
        return frames[d].data_ptr() + f * w * h * 3

    res = {"config": a.config, "members": len(devs), "devices": devs,
           "force_sys": bool(os.environ.get("CAIRO_GROUP_FORCE_SYS"))}
    # one context with the same share of the device as one member
    ctx = cairo_amd.Context(w, h, ring, device=devs[0])
    share = devs.count(devs[0])
    ctx.set_workgroups(max(1, ctx.max_workgroups() // share))
    bench.run_hot_path(ctx, lambda f: ptr(devs[0], f), 0, 32, q, ctx.stages)
    ctx.sync()
    t0 = time.perf_counter()
    bench.run_hot_path(ctx, lambda f: ptr(devs[0], f), 32, a.frames, q, ctx.stages)
    ctx.sync()
    res["one_context_share_mpix"] = round(w * h * a.frames / (time.perf_counter() - t0) / 1e6, 1)
    ctx.close()
    g = cairo_amd.Group(w, h, ring, devs)

    def run(first, count):
        inflight = []
        for f in range(first, first + count):
            if len(inflight) >= g.size * 48:
                t = inflight.pop(0)
                g.wait(t, copy=False)
                g.release(t)
            g.submit(ptr(devs[f % g.size], f), f, f > 0, q, on_device=True)
            inflight.append(f)
        for t in inflight:
            g.wait(t, copy=False)
            g.release(t)

    run(0, 32)
    for m in g.members:
        m.sync()
    t0 = time.perf_counter()
    run(32, a.frames)
    for m in g.members:
        m.sync()
    res["group_mpix"] = round(w * h * a.frames / (time.perf_counter() - t0) / 1e6, 1)
    g.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
