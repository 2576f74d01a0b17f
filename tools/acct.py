"""Steady-state time accounting of the engine's workers (diagnostic).

Needs a library built with CAIRO_ACCT=1 (tools/build_variant.sh acct
-DCAIRO_ACCT=1, copied over cairo_amd/_lib/libcairo_amd.so on the GPU box).
Runs bench.py's timed configuration (default frames per launch, overlapping
launches, feed outputs, frames resident in HBM), zeroes the counters after the
warm-up and prints where the row coders' and row helpers' time goes, per
macroblock / per inter group, summed over every task of the measured launches
(kernels.h Acct).
usage: python tools/acct.py [--config 4k] [--steps 10] [--warmup 3]
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--json", default="")
    ap.add_argument("--helpers", type=int, default=0, help="helper workgroups of a launch (0 = default)")
    a = ap.parse_args()
    import numpy as np
    import torch

    import cairo_amd

    w, h, ring, q, _ = bench.CONFIGS[a.config]
    batch = cairo_amd.default_batch(w, h)
    warm, timed = a.warmup * batch, a.steps * batch
    n = warm + timed
    frames = torch.empty((n, h, w, 3), dtype=torch.uint8, device="cuda:0")
    for f in range(n):
        frames[f].copy_(torch.from_numpy(cairo_amd.make_band4(w, h, f)))
    torch.cuda.synchronize()
    base, stride = frames.data_ptr(), w * h * 3
    ctx = cairo_amd.Context(w, h, ring)
    ctx.set_outputs(cairo_amd.OUT_FEED)
    ctx.set_debug(32)
    if a.helpers:
        ctx.set_helpers(a.helpers)
    bench.run_hot_path(ctx, lambda f: base + f * stride, 0, warm, q, ctx.stages)
    ctx.sync()
    ctx.read_acct(reset=True)
    t0 = time.perf_counter()
    bench.run_hot_path(ctx, lambda f: base + f * stride, warm, timed, q, ctx.stages)
    ctx.sync()
    el = time.perf_counter() - t0
    c = ctx.read_acct()
    ctx.close()
    us = lambda ticks: ticks / 100.0  # noqa: E731  (10 ns ticks)
    mbs = max(c["coder_mbs"], 1)
    groups = max(c["helper_tasks"] * ((w + 63) // 64), 1)
    parts = ("group_wait", "window", "search", "inter", "xform", "publish", "drain", "vm0", "records", "prebarrier",
             "store_tail")
    coder = {k: round(us(c["coder_" + k]) / mbs, 3) for k in ("total",) + parts}
    coder["rest"] = round(coder["total"] - sum(coder[k] for k in parts), 3)
    coder["dequeue_per_task"] = round(us(c["coder_dequeue"]) / max(c["coder_tasks"], 1), 2)
    # inside "search": thread 0's wave per stage phase (evaluation + LDS stores, barrier, LDS reads + replay)
    coder["search_phases"] = {k: round(us(c[k]) / mbs, 3) for k in
                              ("search_eval", "search_barrier", "search_select", "subpel_eval", "subpel_barrier",
                               "subpel_select")}
    helper = {k: round(us(c["helper_" + k]) / groups, 3) for k in ("total", "wait", "deblock", "search", "catchup")}
    helper["rest"] = round(helper["total"] - sum(helper[k] for k in ("wait", "deblock", "search", "catchup")), 3)
    helper["dequeue_per_task"] = round(us(c["helper_dequeue"]) / max(c["helper_tasks"], 1), 2)
    helper["deblock_phases"] = {k: round(us(c[k]) / groups, 3) for k in ("db_inputs", "db_filter", "db_write")}
    helper["chunks_per_group"] = round(c["helper_chunks"] / groups, 3)
    mb = 1e6
    traffic = {k: round(c[k] / timed / mb, 2) for k in
               ("win_bytes", "win_spec_unused_bytes", "zero_mv_bytes", "gran_poll_bytes", "rec_poll_bytes")}
    traffic["unit"] = "MB per frame (requested)"
    traffic["searched_task_frac"] = round(c["searched_tasks"] / max(c["inter_tasks"], 1), 3)
    traffic["win_stages_per_frame"] = round(c["win_stages"] / timed, 1)
    out = {"config": a.config, "timed_frames": timed, "mpix_s": round(w * h * timed / el / 1e6, 1),
           "coder_us_per_mb": coder, "helper_us_per_group": helper, "traffic": traffic, "raw": c}
    print(json.dumps(out))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
