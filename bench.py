"""bench.py -- encoded Mpixels/s of the EVX-1 encode hot path on MI355X.

Metric (BASELINE.json): encoded Mpixels/s (p-frame, q=16), bit-exact vs ref.
Workload (BASELINE.json configs[1]): 1280x720, p-frame with 1 reference
(ring R = 2), quality 16, band4 synthetic content (seed 1234).

A step = one P-frame through the hot path: RGB->YUV, inter search, the
macroblock wavefront (intra search, classify, transform, VAQ, quantize,
reconstruct, in-loop deblock), and the block table + coefficients handed to host
memory for the entropy stage.  All input frames are resident in HBM before the
timed region.  The host entropy stage (outside the hot path by design) is
measured separately (end_to_end) and the output is checked bit-exact against
the oracle on the cpu_baseline sample.

Multi-GPU: one process per GPU (torch.distributed.run); every rank encodes its
own stream (the path has no cross-stream exchange), value = aggregate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import deque

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (width, height, ring, quality, BASELINE.json configs index)
    "720p": (1280, 720, 2, 16, 1),
    "1080p": (1920, 1080, 4, 8, 2),
    "4k": (3840, 2160, 4, 16, 3),
    "cif": (352, 288, 4, 16, 0),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=300, help="timed P-frames (BASELINE configs: 300-frame IPPP streams)")
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="720p", choices=sorted(CONFIGS))
    p.add_argument("--cpu-frames", type=int, default=0,
                   help="P-frames in the bounded CPU baseline sample (0 = about 60 Mpixels: 10-20 s of one core)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--entropy-threads", type=int, default=0,
                   help="entropy workers per rank (0: min(14, host CPUs / ranks - 2); the GPU box gives 16 CPUs per GPU)")
    p.add_argument("--no-end-to-end", action="store_true")
    p.add_argument("--pmc", default=None, help="PMC summary json (profiles/) for roofline.traffic")
    p.add_argument("--batch", type=int, default=0, help="frames per engine launch (pipelined; 0 = library default)")
    p.add_argument("--rows", type=int, default=0, help="row-coder (= helper) workgroups per launch (0 = library default)")
    return p.parse_args()


def algorithmic_bytes(w, h, ring):
    """bytes per frame, P = one int16 YUV420 plane set."""
    wa, ha = (w + 15) & ~15, (h + 15) & ~15
    P = 3 * wa * ha
    return {
        "convert": 3 * w * h + P,
        # inter search (source + R-1 references), row coding (source, slot
        # window, prediction, recon + coefficient writes), deblock (read + write)
        "engine": ring * P + 5 * P + 2 * P,
    }


def max_over_ranks(x: float, dist, device) -> float:
    """Max of a per-rank float over the process group (identity without one).
    device: where the collective's tensor lives (cuda for nccl, cpu for gloo)."""
    if dist is None:
        return x
    import torch

    t = torch.tensor([x], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_mpix(w: int, h: int, steps: int, world: int, elapsed_max: float) -> float:
    """Whole-job throughput: every rank encodes `steps` frames of w x h (weak scaling)."""
    return w * h * steps * world / elapsed_max / 1e6


def run_hot_path(ctx, dev_frames, frame_ptr, first, count, quality, stages, entropy=None):
    """Submit frames [first, first+count) with up to `stages` in flight."""
    inflight = deque()
    for f in range(first, first + count):
        if len(inflight) == stages:
            t = inflight.popleft()
            out = ctx.wait(t, copy=False)
            if entropy is not None:
                entropy(t, out)
            else:
                ctx.release(t)
        inflight.append(ctx.submit(frame_ptr(f), f, f > 0, quality, on_device=True))
    while inflight:
        t = inflight.popleft()
        out = ctx.wait(t, copy=False)
        if entropy is not None:
            entropy(t, out)
        else:
            ctx.release(t)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch  # device memory, barrier and max-over-ranks timing only

    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import cairo_amd

    w, h, ring, q, cfg_idx = CONFIGS[a.config]
    nframes = a.warmup + a.steps
    # synthetic input, uploaded to HBM before timing
    host = np.empty((nframes, h, w, 3), np.uint8)
    for f in range(nframes):
        host[f] = cairo_amd.make_band4(w, h, f)
    frames = torch.from_numpy(host).to(dev)
    base, stride = frames.data_ptr(), w * h * 3

    def frame_ptr(f):
        return base + f * stride

    ctx = cairo_amd.Context(w, h, ring, device=local)
    if a.batch:
        ctx.set_batch(a.batch)
    if a.rows:
        ctx.set_workgroups(a.rows)
    stages = ctx.L.cairo_ctx_stages(ctx.h)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    # warmup: frame 0 (I) + P-frames 1..W-1
    run_hot_path(ctx, frames, frame_ptr, 0, a.warmup, q, stages)
    ctx.sync()
    ctx.set_profiling(True)
    ctx.take_timings()
    barrier()
    t0 = time.perf_counter()
    run_hot_path(ctx, frames, frame_ptr, a.warmup, a.steps, q, stages)
    ctx.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms, kframes = ctx.take_timings()
    ctx.set_profiling(False)
    elapsed = max_over_ranks(elapsed, dist, dev)
    value = aggregate_mpix(w, h, a.steps, world, elapsed)
    # per-frame kernel time: the engine encodes a batch of frames per launch
    per_kernel = {"convert": kernel_ms[0] / max(kframes, 1), "engine": kernel_ms[2] / max(kframes, 1)}
    abytes = algorithmic_bytes(w, h, ring)
    dominant = max(per_kernel, key=per_kernel.get)

    def roofline(kernel):
        ms = per_kernel[kernel]
        ach = abytes[kernel] / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        return {"kernel": kernel, "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": None, "algorithmic_bytes": abytes[kernel],
                "avg_ms": round(ms, 4), "per": "frame (engine launches cover a batch of frames)"}

    roof = roofline(dominant)
    pmc_path = a.pmc or os.path.join(ROOT, "profiles", f"pmc_{a.config}.json")
    if os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path))
        k = pmc.get("per_frame_hbm_bytes", {}).get(roof["kernel"])
        if k is not None:
            roof["traffic"] = k
            roof["traffic_source"] = os.path.relpath(pmc_path, ROOT)
        ws = pmc.get("engine_wave_states")
        if ws and roof["kernel"] == "engine":
            # SQ counters of the same workload: where the engine's wave time goes
            # (the kernel is dependency-latency-bound, not HBM-bound)
            roof["wave_states"] = {k2: round(ws[k2], 3) for k2 in
                                   ("waiting_frac", "issue_stalled_frac", "issuing_frac", "valu_issue_frac_of_chip")
                                   if k2 in ws}

    # end-to-end: hot path + host entropy on worker threads (rank 0 reports)
    e2e = None
    if not a.no_end_to_end:
        ctx2 = cairo_amd.Context(w, h, ring, device=local)
        if a.batch:
            ctx2.set_batch(a.batch)
        e2e = end_to_end(cairo_amd, ctx2, frame_ptr, a, ring, q, w, h, barrier, dist, dev, world)
        ctx2.close()

    result = {
        "metric": "encoded Mpixels/s (p-frame, q=16) at 1/2/4/8 MI355X; bit-exact vs ref",
        "value": round(value, 3),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed * 1e3 / a.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic (band4 generator, seed 1234; SURVEY.md §8(d))",
        "config": {"workload": f"{w}x{h} p-frame q={q} ring R={ring} (BASELINE.json configs[{cfg_idx}])",
                   "width": w, "height": h, "ring": ring, "quality": q,
                   "parallelism": f"replicas: {world} independent stream(s), one per GPU"},
        "roofline": roof,
        "kernels_avg_ms": {k: round(v, 4) for k, v in per_kernel.items()},
        "end_to_end": e2e,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        nf = a.cpu_frames or max(2, min(48, int(60e6 / (w * h))))
        result["cpu_baseline"], result["bit_exact"] = cpu_baseline(cairo_amd, w, h, ring, q, nf)
    else:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def end_to_end(cairo_amd, ctx, frame_ptr, a, ring, q, w, h, barrier, dist, dev, world):
    """Hot path + host entropy through the native frame pipeline
    (cairo_stream_*: entropy on a pool of C++ worker threads); every frame's
    payload is appended to one output buffer (bitstream produced)."""
    stages = ctx.L.cairo_ctx_stages(ctx.h)
    if a.entropy_threads <= 0:
        a.entropy_threads = max(1, min(14, (os.cpu_count() or 4) // world - 2))
    st = cairo_amd.Stream(ctx, threads=a.entropy_threads)
    out = np.zeros(max(w * h * 4, 1 << 20), np.uint8)  # payload bits of the frames in flight, reused

    tl = []

    def collect(tk):
        st.collect(tk, out, 0)
        tl.append(st.timeline(tk))

    def run(first, count):
        inflight = deque()
        for f in range(first, first + count):
            if len(inflight) == stages:
                collect(inflight.popleft())
            inflight.append(st.submit(frame_ptr(f), f, f > 0, q, on_device=True))
        while inflight:
            collect(inflight.popleft())

    run(0, a.warmup)  # I + P warmup
    barrier()
    t0 = time.perf_counter()
    tl.clear()
    run(a.warmup, a.steps)
    barrier()
    el = time.perf_counter() - t0
    st.close()
    el = max_over_ranks(el, dist, dev)
    T = np.array(tl)  # per frame: submitted, outputs on host, entropy start/end, collected (us)
    mid = T[len(T) // 4: 3 * len(T) // 4]
    pipeline = {
        "latency_submit_to_outputs_ms": round(float(np.mean(T[:, 1] - T[:, 0])) / 1e3, 3),
        "entropy_ms_per_frame_per_thread": round(float(np.mean(T[:, 3] - T[:, 2])) / 1e3, 3),
        "steady_period_ms_per_frame": round(float(np.mean(np.diff(mid[:, 4]))) / 1e3, 4),
    }
    return {"value": round(aggregate_mpix(w, h, a.steps, world, el), 3), "unit": "Mpix/s",
            "ms_per_step": round(el * 1e3 / a.steps, 4), "entropy_threads": a.entropy_threads,
            "staging_slots": stages, "pipeline": pipeline,
            "note": "hot path + host entropy (native frame pipeline, cairo_stream_*); payload bits produced"}


def cpu_baseline(cairo_amd, w, h, ring, q, pframes):
    """The oracle (plain-C restatement of the reference encoder, test
    infrastructure) on one host core over a bounded sample: frame 0 (I) +
    `pframes` P-frames; P-frame Mpix/s.  The same frames are then encoded by
    the GPU path + host entropy and compared bit for bit (the checker role)."""
    from oracle import oracle as orc

    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    ref = []
    tp = 0.0
    for t in range(pframes + 1):
        rgb = cairo_amd.make_band4(w, h, t)
        t0 = time.perf_counter()
        data, n = e.encode(rgb)
        dt = time.perf_counter() - t0
        if t > 0:
            tp += dt
        ref.append(orc.canonical_frame_bytes(data, n, t == 0))
    base = {"value": round(w * h * pframes / tp / 1e6, 4), "unit": "Mpix/s", "cores": 1, "kind": "port",
            "sample": f"{w}x{h} q={q} R={ring}: frame 0 (I, untimed) + {pframes} P-frames timed, band4 seed 1234, "
                      f"oracle/evx_oracle.c -O2, one thread"}
    try:
        import platform

        base["cpu"] = platform.processor() or open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": ")
    except Exception:
        pass
    # bit-exact check of the GPU path on the same frames (drop-in encoder API)
    enc = cairo_amd.Encoder(ring=ring)
    enc.set_quality(q)
    bs = cairo_amd.BitStream(w * h * 64)
    mism = []
    for t in range(pframes + 1):
        bs.empty()
        enc.encode(cairo_amd.make_band4(w, h, t), bs)
        if orc.canonical_frame_bytes(bs.data(), bs.bits(), t == 0) != ref[t]:
            mism.append(t)
    enc.close()
    exact = {"frames_checked": pframes + 1, "mismatched_frames": mism, "bit_exact": not mism}
    return base, exact


if __name__ == "__main__":
    main()
