"""bench.py -- encoded Mpixels/s of the EVX-1 encode hot path on MI355X.

Metric (BASELINE.json): encoded Mpixels/s (p-frame, q=16), bit-exact.
Workload (default, BASELINE.json configs[3] on one GPU): 3840x2160 P-frames,
ring R = 4 (3 inter references), quality 16, band4 synthetic content
(seed 1234).  --config 720p / 1080p run configs[1] / configs[2].

A step = one engine launch's batch of P-frames (the library's default frames
per launch: 32 at every bench size) through the hot path: RGB->YUV, inter
search, the macroblock wavefront (intra search, classify, transform, VAQ,
quantize, reconstruct, in-loop deblock), the entropy precode, and each
frame's block table + feed bits handed to host memory for the arithmetic
coder.  --steps 20 therefore times 640 frames after 96 warm-up frames.  All
input frames are resident in HBM before the timed region.  --content noise
/ static run SURVEY.md §8(d)'s stress and best cases instead of band4.

Every frame is verified (bit_exact in the line): each frame's GPU-precoded
feed is copied out of its staging slot as it is retired (the only checking
work inside the timed region), and after timing it is arithmetic-coded on
host threads into the frame's stream record, whose FNV-1a-64 is compared with
tests/golden/stream_<config>_q<q>_r<R>.json (the oracle's per-frame record
hashes of the same band4 stream, made by tests/golden/make_stream_golden.py).
The end-to-end leg's payloads are checked the same way.

Other legs (rank 0, N = 1), outside the timed region:
  end_to_end  hot path + host entropy on native worker threads (cairo_stream)
  api_encode  evx1_encoder::encode() through the drop-in C++ API, called by a
              C++ program built against include/evx1.h (one frame per call,
              host RGB in, bitstream out: the reference's own interface)
  cpu_baseline  the oracle (C restatement) on one host core over a bounded
              sample; the same frames re-check the golden file's prefix and,
              for content without a golden (noise, static), the GPU records

Multi-GPU: one process per GPU (torch.distributed.run).  value (N > 1): ONE
stream over all ranks (BASELINE.json configs[3]: one 4K stream over the
node), frame-interleaved (rank k encodes frames n = k mod N, reading the
others' reconstructions, mirrored into its own memory over xGMI; strong
scaling over the same frames as N = 1); replicas (every rank
encodes its own stream, weak scaling) ride along as an extra field.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from collections import deque
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (width, height, ring, quality, BASELINE.json configs index)
    "4k": (3840, 2160, 4, 16, 3),
    "1080p": (1920, 1080, 4, 8, 2),
    "720p": (1280, 720, 2, 16, 1),
    "cif": (352, 288, 4, 16, 0),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# VALU: 256 CUs x 4 SIMDs x 32 lanes/clock x 2.4 GHz = 78.6 T lane-ops/s
# (MI355X_MICROARCH.md: wave64 issues over 2 clocks); packed 16-bit ops
# (v_sad_u16, v_pk_sub_u16, v_pk_max_u16) do 2 pixel-ops per lane.
VALU_PEAK_PIXEL_OPS = 256 * 4 * 32 * 2.4e9 * 2
# the reference on one Xeon core (P-frame steady state), Mpix/s
REF_CPU_MPIX = {"4k": 1.82, "1080p": 1.61, "720p": 3.56}
API_BIN = os.path.join(ROOT, "cairo_amd", "_lib", "evx1_api_caller")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20, help="timed steps (engine launches of the default batch)")
    p.add_argument("--warmup", type=int, default=3, help="untimed steps before (frame 0 is the I-frame)")
    p.add_argument("--config", default="4k", choices=sorted(CONFIGS))
    p.add_argument("--cpu-frames", type=int, default=0,
                   help="P-frames in the bounded CPU baseline sample (0 = about 60 Mpixels: 10-30 s of one core)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--entropy-threads", type=int, default=0,
                   help="entropy workers per rank (0: min(14, host CPUs / ranks - 2); the GPU box gives 16 CPUs per GPU)")
    p.add_argument("--no-end-to-end", action="store_true")
    p.add_argument("--no-api", action="store_true")
    p.add_argument("--no-single-stream", action="store_true",
                   help="N > 1: skip the frame-interleaved single-stream leg")
    p.add_argument("--pmc", default=None, help="PMC summary json (profiles/) for roofline.traffic")
    p.add_argument("--batch", type=int, default=0, help="frames per engine launch (0 = library default)")
    p.add_argument("--outputs", default="feed", choices=["feed", "coef"],
                   help="what the timed context hands to the host: the GPU-precoded feed (the pipeline's mode) "
                        "or the coefficient planes")
    p.add_argument("--helpers", type=int, default=0, help="helper workgroups of a launch's workers (0 = default)")
    p.add_argument("--rows", type=int, default=0, help="row-coder (= helper) workgroups per launch (0 = library default)")
    p.add_argument("--stages", type=int, default=0, help="staging slots of the timed context (0 = library default)")
    p.add_argument("--intervals", default=None,
                   help="write the timed engine launches' [start, end) intervals (CSV, ms) to this path")
    p.add_argument("--no-host-rgb", action="store_true", help="skip the pipelined host-RGB (PCIe-inclusive) leg")
    p.add_argument("--host-rgb-steps", type=int, default=12, help="timed steps of the host-RGB leg")
    p.add_argument("--content", default="band4", choices=["band4", "noise", "static"],
                   help="band4 (SURVEY.md §8(d) default), noise (no copy blocks, full searches everywhere: the stress "
                        "case) or static (band4 frame 0 repeated: the best case)")
    p.add_argument("--no-verify", action="store_true",
                   help="skip the per-frame check of every timed frame (no feed copies in the timed region)")
    return p.parse_args()


# Frames of one content kind resident in HBM: band4 is a distinct frame per
# index (the golden stream); noise cycles a pool of distinct random frames
# (consecutive frames stay uncorrelated); static is one frame.
NOISE_POOL = 64


def content_frame(kind: str, w: int, h: int, t: int) -> np.ndarray:
    """Source frame t of the bench's stream (RGB888)."""
    import cairo_amd

    if kind == "band4":
        return cairo_amd.make_band4(w, h, t)
    if kind == "static":
        return cairo_amd.make_band4(w, h, 0)
    rng = np.random.default_rng(7 * 1000003 + t % NOISE_POOL)  # tests/content.py "noise"
    return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)


def content_pool(kind: str, frames: int) -> int:
    """Distinct resident frames needed for a stream of `frames` frames."""
    return {"band4": frames, "noise": min(frames, NOISE_POOL), "static": 1}[kind]


class Arena:
    """Append-only host store for per-frame bytes (feeds, payloads): large
    chunks, pre-touched before the timed region, so retiring a frame costs
    one memcpy and no allocation."""

    def __init__(self, chunk: int = 256 << 20):
        self.chunk = chunk
        self.chunks = []
        self.cur, self.pos = -1, 0

    def _new(self, size: int) -> None:
        c = np.empty(size, np.uint8)
        c.fill(0)  # touch every page now, not at the first copy
        self.chunks.append(c)

    def grow(self, nbytes: int) -> None:
        """Pre-touch chunks until about nbytes more fit."""
        free = (self.chunks[self.cur].size - self.pos if self.cur >= 0 else 0) + \
            sum(c.size for c in self.chunks[self.cur + 1:])
        while free < nbytes:
            self._new(self.chunk)
            free += self.chunk

    def reserve(self, nbytes: int):
        """-> (chunk array, byte offset) of nbytes of room (16-byte aligned)."""
        while self.cur < 0 or self.pos + nbytes > self.chunks[self.cur].size:
            if self.cur + 1 == len(self.chunks):
                self._new(max(self.chunk, nbytes))
            self.cur, self.pos = self.cur + 1, 0
        off = self.pos
        self.pos = (off + nbytes + 15) & ~15
        return self.chunks[self.cur], off


class FrameStore:
    """Every frame a leg encodes, kept for the post-timing check: the
    GPU-precoded feed (copied out of the staging slot at retire) or, for the
    end-to-end leg, the payload; a frame whose feed overflowed is coded on
    the spot from its planes (rare: 4K noise at q=1)."""

    def __init__(self):
        self.arena = Arena()
        self.items = {}  # frame -> ("feed" | "pay", chunk, offset, bits) or ("bytes", data, bits)
        self.max_bytes = 0

    def keep_feed(self, cairo_amd, ctx, f, out, ticket):
        if out.feed_status == cairo_amd.FEED_VALID:
            src = out.feed.view(np.uint8)
            buf, off = self.arena.reserve(src.size)
            buf[off:off + src.size] = src
            self.items[f] = ("feed", buf, off, out.feed_bits)
            self.max_bytes = max(self.max_bytes, src.size)
        else:
            self.items[f] = ("bytes",) + payload(cairo_amd, ctx, out, ticket)

    def keep_payload(self, st, f, tk):
        nb = st.payload_bits(tk)
        buf, off = self.arena.reserve(nb // 8 + 8)
        st.collect(tk, buf[off:], 0)
        self.items[f] = ("pay", buf, off, nb)
        self.max_bytes = max(self.max_bytes, nb // 8 + 8)

    def reserve_for(self, frames: int) -> None:
        """Pre-touch room for `frames` more frames of the size seen so far."""
        if self.max_bytes:
            self.arena.grow(int(self.max_bytes * 1.25 + 64) * frames)

    def payload(self, cairo_amd, f):
        it = self.items[f]
        if it[0] == "bytes":
            return it[1], it[2]
        kind, buf, off, nb = it
        if kind == "feed":
            words = buf[off:off + (nb + 31) // 32 * 4].view(np.uint32)
            return cairo_amd.serialize_feed(words, nb)
        return buf[off:off + (nb + 7) // 8].tobytes(), nb


def frame_hashes(cairo_amd, store: FrameStore, w, h, ring, q, threads: int) -> dict:
    """{frame: FNV-1a-64 hex of the canonical stream record} for every frame in
    the store, as tests/golden/make_stream_golden.py hashes the oracle's (the
    arithmetic coding of the feeds runs on `threads` host threads; checker
    code, after the timed region)."""
    from oracle import oracle as orc

    def one(f):
        data, nb = record(cairo_amd, w, h, ring, q, f, *store.payload(cairo_amd, f))
        return f, f"{orc.fnv1a64(orc.canonical_frame_bytes(data, nb, f == 0)):016x}"

    with ThreadPoolExecutor(max(1, threads)) as pool:
        return dict(pool.map(one, sorted(store.items)))


def golden_stream(config: str, content: str, q: int, ring: int):
    """The oracle's per-frame record hashes of this stream, or None."""
    sfx = "" if content == "band4" else f"_{content}"
    path = os.path.join(ROOT, "tests", "golden", f"stream_{config}_q{q}_r{ring}{sfx}.json")
    if not os.path.exists(path):
        return None
    g = json.load(open(path))
    g["path"] = os.path.relpath(path, ROOT)
    return g


def check_hashes(hashes: dict, golden, frames, timed_from: int) -> dict:
    """Compare {frame: hash} for `frames` against the golden file."""
    frames = list(frames)
    have = golden["frame_fnv1a64"] if golden else []
    checked = [f for f in frames if f < len(have)]
    mism = [f for f in checked if hashes.get(f) != have[f]]
    return {"frames": len(frames), "frames_checked": len(checked),
            "timed_frames_checked": sum(1 for f in checked if f >= timed_from),
            "unchecked_frames": len(frames) - len(checked), "mismatched_frames": mism[:50],
            "mismatches": len(mism)}


def algorithmic_bytes(w, h, ring):
    """HBM bytes per frame, P = one int16 YUV420 plane set."""
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


def aggregate_mpix(w: int, h: int, frames: int, world: int, elapsed_max: float) -> float:
    """Whole-job throughput: every rank encodes `frames` frames of w x h (weak scaling)."""
    return w * h * frames * world / elapsed_max / 1e6


def headline(world: int, replicas: dict, single: dict | None) -> dict:
    """The line's value at N GPUs: N = 1, the one context's stream; N > 1,
    the one stream over all ranks (single_stream, strong scaling: the metric
    of BASELINE.json configs[3]), unless that leg failed or was skipped --
    then the replicas' aggregate, labelled as such (weak scaling).
    replicas = {"value", "ms_per_step"}; -> {"value", "scaling", "value_source",
    "ms_per_step"}."""
    if world == 1:
        return {"value": replicas["value"], "scaling": "weak", "value_source": "one stream on one GPU",
                "ms_per_step": replicas["ms_per_step"]}
    if single and single.get("value") is not None and not single.get("error"):
        return {"value": single["value"], "scaling": "strong",
                "value_source": f"single_stream: one stream over {world} GPUs (frame-interleaved group)",
                "ms_per_step": single["ms_per_step"]}
    why = (single or {}).get("error") or "single-stream leg skipped"
    return {"value": replicas["value"], "scaling": "weak",
            "value_source": f"replicas: {world} independent streams (single_stream unavailable: {why})"[:400],
            "ms_per_step": replicas["ms_per_step"]}


def single_stream_check_frames(world: int, ring: int, warm: int) -> int:
    """Frames of the single-stream leg compared with the oracle: at least 2N
    + R, so that every member's frames (each member twice) and every mirror
    push (a frame's reconstruction is pushed to the members of its next R
    frames) are compared; at least 8; at most the warm-up frames."""
    return min(max(2 * world + ring, 8), warm)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def host_cpus() -> int:
    """CPUs this process may use (the GPU box's container quota, not the host's count)."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            return max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    return len(os.sched_getaffinity(0))


def frame_header(w, h, ring, q, t, intra):
    """The stream bytes encode() writes before frame t's payload: the 14-byte
    header on the first frame (byte 7 = 0), then the 10-byte frame descriptor
    (evx1enc.cpp:104-131, common.h:50-76)."""
    import struct

    hdr = struct.pack("<4sHBxHHH", b"EVX1", 14, ring, (2 << 8) | 47, w, h) if t == 0 else b""
    return hdr + struct.pack("<IIH", 0 if intra else 1, t, q)


def record(cairo_amd, w, h, ring, q, t, payload, nbits):
    """Frame t's stream record (header/descriptor + payload) -> (bytes, bits)."""
    head = frame_header(w, h, ring, q, t, t == 0)
    buf = np.zeros(len(head) + len(payload) + 16, np.uint8)
    pos = cairo_amd.bits_append(buf, 0, head, len(head) * 8)
    pos = cairo_amd.bits_append(buf, pos, payload, nbits)
    return buf[: (pos + 7) // 8].tobytes(), pos


def payload(cairo_amd, ctx, out, ticket=None):
    """A frame's payload (bytes, bits) from the context's outputs: the host
    arithmetic coder over the GPU-precoded feed (or the host precode from the
    planes when the feed overflowed)."""
    if out.feed_status == cairo_amd.FEED_VALID:
        return cairo_amd.serialize_feed(out.feed, out.feed_bits)
    cy, cu, cv = (out.coef_y, out.coef_u, out.coef_v) if out.coef_y is not None else ctx.fetch_coef(ticket)
    return cairo_amd.serialize_slice(out.table, ctx.wmb, ctx.hmb, ctx.ring, cy, cu, cv)


def run_hot_path(ctx, frame_ptr, first, count, quality, stages, on_frame=None, on_device=True):
    """Submit frames [first, first+count) with up to `stages` in flight;
    on_frame(index, outputs) sees a frame's outputs before its release.
    frame_ptr(f): a device address (on_device), or a host frame the context
    uploads at submit."""
    inflight = deque()

    def retire():
        f, t = inflight.popleft()
        out = ctx.wait(t, copy=False)
        if on_frame is not None:
            on_frame(f, out, t)
        ctx.release(t)

    for f in range(first, first + count):
        if len(inflight) == stages:
            retire()
        inflight.append((f, ctx.submit(frame_ptr(f), f, f > 0, quality, on_device=on_device)))
    while inflight:
        retire()


T_START = time.perf_counter()


def note(rank, msg):
    """Progress on stderr (the JSON line stays the only stdout line)."""
    print(f"[bench rank {rank} +{time.perf_counter() - T_START:.0f}s] {msg}", file=sys.stderr, flush=True)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch  # device memory, barrier and max-over-ranks timing only

    dist = None
    if world > 1:
        import torch.distributed as dist

    # Rehearsal of the multi-rank paths on a one-GPU box (tests, never the
    # driver's runs): CAIRO_BENCH_SHARED_DEVICE=1 puts every rank on device 0,
    # over gloo (RCCL refuses two ranks on one GPU), each with its share of
    # the workgroup slots.
    shared = world > 1 and os.environ.get("CAIRO_BENCH_SHARED_DEVICE") == "1"
    if shared:
        local = 0
    if world > 1:
        dist.init_process_group("gloo" if shared else "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cpu") if shared else torch.device("cuda", local)  # where collectives' tensors live

    def share(c):  # ranks sharing one device split its resident workgroup slots
        if shared:
            c.set_workgroups(max(1, c.max_workgroups() // world))
        return c

    import cairo_amd

    w, h, ring, q, cfg_idx = CONFIGS[a.config]
    batch = a.batch or cairo_amd.default_batch(w, h)
    warm_frames, timed_frames = a.warmup * batch, a.steps * batch
    nframes = warm_frames + timed_frames
    # the end-to-end leg encodes twice the timed frames after the same warm-up:
    # every frame of every leg is a distinct resident frame of one stream, the
    # one the golden hashes describe (4K: 1376 frames, 34 GB of HBM)
    stream_frames = warm_frames + (timed_frames if a.no_end_to_end else 2 * timed_frames)
    pool_n = content_pool(a.content, max(nframes, stream_frames))
    # synthetic input, generated on host threads and uploaded to HBM before timing
    frames = torch.empty((pool_n, h, w, 3), dtype=torch.uint8, device=torch.device("cuda", local))
    chunk = 16
    with ThreadPoolExecutor(max(1, min(8, host_cpus()))) as pool:
        for c0 in range(0, pool_n, chunk):
            n = min(chunk, pool_n - c0)
            host = np.stack(list(pool.map(lambda f: content_frame(a.content, w, h, f), range(c0, c0 + n))))
            frames[c0:c0 + n].copy_(torch.from_numpy(host))
    torch.cuda.synchronize()
    base, stride = frames.data_ptr(), w * h * 3
    note(rank, f"{pool_n} {w}x{h} {a.content} frames resident in HBM")

    def frame_ptr(f):
        return base + (f % pool_n) * stride

    ctx = share(cairo_amd.Context(w, h, ring, device=local, **({"stages": a.stages} if a.stages else {})))
    ctx.set_batch(batch)
    # what the pipeline and the drop-in encoder hand to the host coder
    ctx.set_outputs(cairo_amd.OUT_FEED if a.outputs == "feed" else cairo_amd.OUT_COEF)
    if a.rows:
        ctx.set_workgroups(a.rows)
    if a.helpers:
        ctx.set_helpers(a.helpers)
    stages = ctx.stages

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    # the oracle's live sample (rank 0, N = 1): the CPU baseline's frames;
    # without a golden file (noise, static) also every frame of the first
    # launch and the head of the second
    check = rank == 0 and world == 1 and not a.no_cpu_baseline
    golden = golden_stream(a.config, a.content, q, ring)
    # CPU baseline: frame 0 + a bounded sample of P-frames (about 60 Mpixels)
    cpu_pframes = a.cpu_frames or max(2, min(48, int(60e6 / (w * h))))
    n_check = (cpu_pframes + 1 if golden else max(cpu_pframes + 1, batch + 3)) if check else 0
    n_check = min(n_check, warm_frames)
    verify = not a.no_verify
    hot = FrameStore()

    def keep(f, out, ticket):
        hot.keep_feed(cairo_amd, ctx, f, out, ticket)

    # warmup: frame 0 (I) + P-frames, in the same context and launches as the timed region
    run_hot_path(ctx, frame_ptr, 0, warm_frames, q, stages, keep if verify or n_check else None)
    ctx.sync()
    hot.reserve_for(timed_frames)
    note(rank, "warm-up done")
    ctx.set_profiling(True)
    ctx.take_timings()
    barrier()
    t0 = time.perf_counter()
    run_hot_path(ctx, frame_ptr, warm_frames, timed_frames, q, stages, keep if verify else None)
    ctx.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    intervals = ctx.busy_intervals()
    kernel_ms, kframes = ctx.take_timings()
    launches = max(1, a.steps)
    if a.intervals and rank == 0:
        with open(a.intervals, "w") as fh:
            fh.write(f"# {w}x{h} R={ring} q={q}: timed k_engine launches, {batch} frames each, {timed_frames} frames; "
                     f"[start, end) ms on one HIP-event clock (launch streams)\n")
            fh.write("launch,start_ms,end_ms,frames\n")
            for i, (s0, s1) in enumerate(intervals):
                fh.write(f"{i},{s0:.4f},{s1:.4f},{batch}\n")
    ctx.set_profiling(False)
    elapsed = max_over_ranks(elapsed, dist, dev)
    value = aggregate_mpix(w, h, timed_frames, world, elapsed)
    note(rank, f"timed region: {timed_frames} frames in {elapsed:.3f} s")
    replicas = {"value": round(value, 3), "unit": "Mpix/s", "scaling": "weak", "streams": world,
                "ms_per_step": round(elapsed * 1e3 / a.steps, 4), "ms_per_frame": round(elapsed * 1e3 / timed_frames, 4),
                "timed_frames_per_rank": timed_frames,
                "note": "every rank encodes its own stream (independent replicas); whole-job aggregate"}
    kf = max(kframes, 1)
    abytes = algorithmic_bytes(w, h, ring)
    engine_busy_ms = kernel_ms[3] / kf  # union of the launch intervals / frames
    roof = {
        "kernel": "k_engine", "bound": "hbm",
        "achieved": round(abytes["engine"] / (engine_busy_ms * 1e-3) / 1e9, 2),
        "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": None, "traffic": None,
        "algorithmic_bytes": abytes["engine"], "per": "frame",
        "engine_busy_ms_per_frame": round(engine_busy_ms, 4),
        "avg_launch_ms": round(kernel_ms[2] / launches, 3), "frames_per_launch": batch,
        "launches": int(len(intervals)),
        "note": "achieved = SURVEY §8(d) algorithmic bytes per frame / (engine busy time / frames); busy time = "
                "union of the k_engine launch intervals (HIP events on the launch streams; two launches overlap, "
                "avg_launch_ms is the per-launch duration rocprofv3 --stats reports)",
    }
    roof["frac"] = round(roof["achieved"] / HBM_PEAK_GBS, 6)
    pmc_path = a.pmc or os.path.join(ROOT, "profiles", f"pmc_{a.config}" +
                                     ("" if a.content == "band4" else f"_{a.content}") + ".json")
    if os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path))
        k = pmc.get("per_frame_hbm_bytes_sized") or pmc.get("per_frame_hbm_bytes", {}).get("engine")
        if k is not None:  # by request size (TCC_EA0_RDREQ_32B/64B/128B, WRREQ) when profiled so
            roof["traffic"] = k
            roof["traffic_source"] = os.path.relpath(pmc_path, ROOT)
        ws = pmc.get("engine_wave_states")
        if ws:
            # SQ counters of the same workload: where the engine's wave time goes
            # (the kernel is dependency-latency-bound, not HBM-bound)
            roof["wave_states"] = {k2: round(ws[k2], 3) for k2 in
                                   ("waiting_frac", "issue_stalled_frac", "issuing_frac", "valu_issue_frac_of_chip")
                                   if k2 in ws}
    ops_path = os.path.join(ROOT, "profiles", "algorithmic_ops.json")
    valu = None
    if os.path.exists(ops_path):
        ops = json.load(open(ops_path)).get(a.config if a.content == "band4" else f"{a.config}_{a.content}")
        if ops:
            per_frame = ops["pixel_ops_per_p_frame"]
            ach = per_frame / (engine_busy_ms * 1e-3)
            valu = {"bound": "valu", "achieved": round(ach / 1e12, 4), "peak": round(VALU_PEAK_PIXEL_OPS / 1e12, 1),
                    "unit": "Tpixel-ops/s", "frac": round(ach / VALU_PEAK_PIXEL_OPS, 5),
                    "pixel_ops_per_frame": per_frame, "source": "profiles/algorithmic_ops.json",
                    "note": "SURVEY §8(d) pixel-ops (256 per SAD, 384 per MAD and per lerp, counted by the oracle "
                            "on band4) / engine busy time; peak = packed 16-bit VALU rate (2 pixel-ops per lane)"}

    e2e = None
    e2e_store = FrameStore() if verify else None
    if not a.no_end_to_end:
        note(rank, "end-to-end leg")
        # the pipeline's depth: two launches in flight hold 2 * batch staging
        # slots, the host entropy works on the rest; 128 (not the library's
        # 96) keeps 64 for it at 32 frames per launch
        ctx2 = share(cairo_amd.Context(w, h, ring, device=local, stages=a.stages or E2E_STAGES))
        ctx2.set_batch(batch)
        # twice the timed leg's frames (all resident, the same stream), so
        # that the last launch's entropy tail weighs half as much
        e2e = end_to_end(cairo_amd, ctx2, frame_ptr, a, ring, q, w, h, warm_frames,
                         2 * timed_frames, barrier, dist, dev, world, e2e_store, batch)
        ctx2.close()
    ctx.close()
    host_leg = None
    if not a.no_host_rgb and world == 1:
        note(rank, "host-RGB leg")
        host_leg = host_rgb(cairo_amd, a, w, h, ring, q, batch, local)
    single = None
    if world > 1 and not a.no_single_stream:
        note(rank, "single-stream leg")
        single = single_stream(cairo_amd, frame_ptr, a, w, h, ring, q, batch, warm_frames, timed_frames, barrier,
                               dist, dev, world, rank, local, share)
    del frames
    torch.cuda.empty_cache()

    api = None
    if rank == 0 and world == 1 and not a.no_api:
        note(rank, "encode() API leg")
        api = api_encode(w, h, ring, q, 2 + max(4, min(12, int(100e6 / (w * h)))))

    head = headline(world, replicas, single)
    where = "on one GPU" if world == 1 else f"as one stream over {world} GPUs"
    result = {
        "metric": "encoded Mpixels/s (p-frame, q=16) at 1/2/4/8 MI355X; bit-exact vs ref",
        "value": head["value"],
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": head["scaling"],
        "value_source": head["value_source"],
        # the reference publishes no number (its CPU figures are
        # the survey's own measurements), so no vs_baseline; the CPU ratios
        # below name their denominators
        "vs_baseline": None,
        "dtype": "int16",
        "data": {"band4": "synthetic (band4 generator, seed 1234; SURVEY.md §8(d)), resident in HBM",
                 "noise": f"synthetic uniform RGB noise ({NOISE_POOL} distinct frames cycled; SURVEY.md §8(d) "
                          f"stress case: no copy blocks), resident in HBM",
                 "static": "synthetic static scene (band4 frame 0 repeated; SURVEY.md §8(d) best case), resident "
                           "in HBM"}[a.content],
        "content": a.content,
        "config": {"workload": f"{w}x{h} p-frame q={q} ring R={ring} (BASELINE.json configs[{cfg_idx}] {where})"
                               + ("" if a.content == "band4" else f", {a.content} content"),
                   "width": w, "height": h, "ring": ring, "quality": q, "frames_per_step": batch,
                   "timed_frames": timed_frames, "ms_per_frame": round(head["ms_per_step"] / batch, 4),
                   "parallelism": "one stream on one GPU" if world == 1 else
                   f"single stream, frame-interleaved over {world} GPUs (member k encodes frames n = k mod {world})"},
        "replicas": replicas if world > 1 else None,
        "roofline": roof,
        "roofline_valu": valu,
        "end_to_end": e2e,
        "host_rgb": host_leg,
        "api_encode": api,
        "single_stream": single,
    }
    exact = None
    if verify or n_check:
        note(rank, "checking every frame")
        tv = time.perf_counter()
        threads = max(1, host_cpus() // world)
        hot_h = frame_hashes(cairo_amd, hot, w, h, ring, q, threads)
        e2e_h = frame_hashes(cairo_amd, e2e_store, w, h, ring, q, threads) if e2e_store and e2e_store.items else {}
        del hot, e2e_store
        exact = {"golden": ({"path": golden["path"], "frames": golden["frames"]} if golden else None)}
        if verify:
            exact["hot_path_context"] = check_hashes(hot_h, golden, range(nframes), warm_frames)
            if e2e_h:
                exact["end_to_end_pipeline"] = check_hashes(e2e_h, golden, range(stream_frames), warm_frames)
        exact["check_s"] = round(time.perf_counter() - tv, 2)
    if check:
        note(rank, "CPU baseline and the oracle's live sample")
        result["cpu_baseline"], sample = cpu_baseline(cairo_amd, a.content, w, h, ring, q, cpu_pframes, n_check - 1,
                                                      hot_h, e2e_h, golden, batch)
        exact["oracle_sample"] = sample
    else:
        result["cpu_baseline"] = None
    if exact is not None:
        hp = exact.get("hot_path_context", {})
        bad = sum(exact.get(k, {}).get("mismatches", 0) for k in ("hot_path_context", "end_to_end_pipeline"))
        bad += len(exact.get("oracle_sample", {}).get("mismatched_frames", []))
        exact["frames_checked"] = hp.get("timed_frames_checked", 0)  # timed frames, against the golden hashes
        exact["timed_frames"] = timed_frames
        exact["mismatches"] = bad
        # true only when every timed frame was compared; a run without a golden
        # stream (only the oracle's live sample of warm-up frames) is unverified
        exact["verified"] = exact["frames_checked"] == timed_frames
        exact["bit_exact"] = False if bad else (True if exact["verified"] else None)
        exact["what"] = ("every frame of the timed context (warm-up and timed, same launches) and of the end-to-end "
                         "pipeline: the GPU feed / payload arithmetic-coded on host threads after the timed region, "
                         "the frame's stream record hashed (FNV-1a-64, header byte 7 and tail bits masked) and "
                         "compared with the oracle's hashes of the same stream (golden); oracle_sample re-encodes "
                         "the first frames live on this host")
    if world > 1:
        allx = [None] * world
        dist.all_gather_object(allx, exact)
        vals = [(x or {}).get("bit_exact") for x in allx]
        exact = {"ranks": allx, "bit_exact": False if False in vals else (None if None in vals else True),
                 "frames_checked": sum((x or {}).get("frames_checked", 0) for x in allx),
                 "what": "every rank's own replica stream, every frame, against the golden hashes"}
    result["bit_exact"] = exact
    vs = {}
    if a.config in REF_CPU_MPIX:
        vs["survey_xeon_reference"] = round(result["value"] / REF_CPU_MPIX[a.config], 1)
    if result["cpu_baseline"]:
        vs["this_box_oracle"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
    result["vs_cpu"] = dict(vs, note="value / a one-core CPU encode: survey_xeon_reference = the reference itself "
                                     "on one Xeon core of the survey container (BASELINE.md, not a published "
                                     "number); this_box_oracle = cpu_baseline.value (the oracle, a C restatement "
                                     "of the reference, on one core of this box)")
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def agreed_step(dist, group, rank, state, what, fn):
    """Run fn unless a rank already failed, then agree on failure over
    `group`: every rank makes the same collective call whatever happened, so
    a rank that failed never leaves the others waiting in a barrier.  state
    ["err"] holds this rank's first error; returns True while all ranks are
    fine."""
    import torch

    if not state["err"]:
        try:
            fn()
        except Exception as ex:  # noqa: BLE001 -- reported in the line
            state["err"] = f"rank {rank} ({what}): {type(ex).__name__}: {ex}"[:300]
            note(rank, f"failed: {state['err']}")
    bad = torch.tensor([1.0 if state["err"] else 0.0], dtype=torch.float64)
    dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=group)
    if bad.item() and not state["err"]:
        state["err"] = f"rank {rank}: stopped ({what}): another rank failed"
    return not state["err"]


def single_stream(cairo_amd, frame_ptr, a, w, h, ring, q, batch, warm, timed, barrier, dist, dev, world, rank,
                  local, share):
    """N > 1: ONE stream over all ranks, frame-interleaved:
    rank k encodes frames n = k (mod N), reading the other ranks'
    reconstructions, output_cache and progress words in place over xGMI
    (IPC handles exchanged over gloo).  Strong scaling: the same frames as
    the N = 1 run, value = stream pixels / max-over-ranks time.  The first
    frames are serialized and compared with the oracle on rank 0.  Failures
    are reported, not raised (the replicas line above stays valid)."""
    import torch

    gloo = dist.new_group(backend="gloo")
    res, err = None, ""
    n_check = single_stream_check_frames(world, ring, warm)
    recs = {}
    ctx = None
    state = {"err": ""}

    def step(what, fn):
        return agreed_step(dist, gloo, rank, state, what, fn)

    store = FrameStore()

    def run(first, count, keep):
        inflight = deque()

        def retire():
            n, t = inflight.popleft()
            out = ctx.wait(t, copy=False)
            if keep:
                store.keep_feed(cairo_amd, ctx, n, out, t)
            ctx.release(t)

        for n in range(first, first + count):
            if n % world != rank:
                continue
            if len(inflight) == ctx.stages:
                retire()
            inflight.append((n, ctx.submit(frame_ptr(n), n, n > 0, q, on_device=True)))
        ctx.flush()
        while inflight:
            retire()
        ctx.sync()

    def make():
        nonlocal ctx
        # the library's staging slots (96): every member imports the others'
        # output_cache over IPC, exported in chunks below 1 GiB each
        ctx = share(cairo_amd.Context(w, h, ring, device=local, **({"stages": a.stages} if a.stages else {})))
        ctx.set_batch(batch)
        ctx.set_outputs(cairo_amd.OUT_FEED)

    info = {}
    step("context", make)
    note(rank, "single stream: context made")
    step("peer info", lambda: info.update(rec=ctx.peer_info(cross_device=True)))
    note(rank, "single stream: peer info")
    peers = [None] * world
    dist.all_gather_object(peers, info.get("rec"), group=gloo)
    note(rank, "single stream: peers gathered")
    # in-kernel waits on other ranks' frames are bounded (2 s): ranks start each phase together
    if step("join", lambda: ctx.join_group(rank, peers)):
        note(rank, "single stream: group joined")
    if step("warm-up", lambda: run(0, warm, True)):
        note(rank, "single stream: warm-up done")
    store.reserve_for(len(range(rank, timed, world)))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if step("timed", lambda: run(warm, timed, not a.no_verify)):
        res = time.perf_counter() - t0
        note(rank, "single stream: timed run done")
    err = state["err"]
    # this member's frames, checked after the timed region: the live oracle's
    # first frames on rank 0 below, every frame against the golden hashes
    mine = {}
    if not err:
        mine = frame_hashes(cairo_amd, store, w, h, ring, q, max(1, host_cpus() // world))
    del store
    golden = golden_stream(a.config, a.content, q, ring)
    gcheck = check_hashes(mine, golden, sorted(mine), warm) if golden else None
    recs = {n: mine[n] for n in mine if n < n_check}
    own = len(range(rank, timed, world))  # this member's frames of the timed region
    per_member = [None] * world
    dist.all_gather_object(per_member, round(res * 1e3 / max(own, 1), 4) if res else None, group=gloo)
    gchecks = [None] * world
    dist.all_gather_object(gchecks, gcheck, group=gloo)
    ok = torch.tensor([0.0 if err else 1.0], dtype=torch.float64)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=gloo)
    elt = torch.tensor([res or 0.0], dtype=torch.float64)
    dist.all_reduce(elt, op=dist.ReduceOp.MAX, group=gloo)
    errs = [None] * world
    dist.all_gather_object(errs, err, group=gloo)
    allrecs = [None] * world
    dist.all_gather_object(allrecs, recs, group=gloo)
    dist.barrier(group=gloo)  # nobody frees buffers another rank may still read
    if ctx is not None:
        ctx.close()
    if ok.item() < 1:
        return {"error": [e for e in errs if e]}
    el = float(elt.item())
    out = {"value": round(aggregate_mpix(w, h, timed, 1, el), 3), "unit": "Mpix/s", "scaling": "strong",
           "members": world, "world_size_seen": dist.get_world_size(),
           "backend": dist.get_backend(), "ms_per_frame": round(el * 1e3 / timed, 4),
           "ms_per_step": round(el * 1e3 / max(1, timed // batch), 4), "timed_frames": timed,
           "member_ms_per_own_frame": per_member,
           "note": "one stream, frame n on rank n % N (frame-interleaved group; each frame's reconstruction "
                   "pushed into the memory of the members that read it); same frames as the N = 1 run"}
    if rank == 0:
        from oracle import oracle as orc

        got = {}
        for r in allrecs:
            got.update(r)
        e = orc.OracleEncoder(ring)
        e.set_quality(q)
        mism = []
        for t in range(n_check):
            data, nb = e.encode(content_frame(a.content, w, h, t))
            if got.get(t) != f"{orc.fnv1a64(orc.canonical_frame_bytes(data, nb, t == 0)):016x}":
                mism.append(t)
        ex = {"oracle_sample": {"frames": n_check, "members_covered": min(world, n_check), "mismatched_frames": mism}}
        bad = len(mism)
        if all(gchecks):
            ex["members_vs_golden"] = gchecks
            ex["frames_checked"] = sum(g["timed_frames_checked"] for g in gchecks)
            bad += sum(g["mismatches"] for g in gchecks)
        ex["mismatches"] = bad
        ex["verified"] = ex.get("frames_checked") == timed
        ex["bit_exact"] = False if bad else (True if ex["verified"] else None)
        out["bit_exact"] = ex
    return out


E2E_STAGES = 128  # staging slots of the end-to-end leg's context


def end_to_end(cairo_amd, ctx, frame_ptr, a, ring, q, w, h, warm, timed, barrier, dist, dev, world, store,
               batch=0):
    """Hot path + host entropy through the native frame pipeline
    (cairo_stream_*: entropy on a pool of C++ worker threads); every frame's
    payload is collected into host memory (store: kept for the post-timing
    check; without one, into one reused buffer)."""
    stages = ctx.stages
    if a.entropy_threads <= 0:
        a.entropy_threads = max(1, min(14, host_cpus() // world - 2))
    st = cairo_amd.Stream(ctx, threads=a.entropy_threads)
    out = np.zeros(max(w * h * 4, 1 << 20), np.uint8)  # payload bits of the frames in flight, reused
    tl = []

    def collect(f, tk):
        if store is not None:
            store.keep_payload(st, f, tk)
        else:
            st.collect(tk, out, 0)
        tl.append(st.timeline(tk))

    def run(first, count):
        inflight = deque()
        for f in range(first, first + count):
            if len(inflight) == stages:
                collect(*inflight.popleft())
            inflight.append((f, st.submit(frame_ptr(f), f, f > 0, q, on_device=True)))
        while inflight:
            collect(*inflight.popleft())

    run(0, warm)  # I + P warmup
    if store is not None:
        store.reserve_for(timed)
    barrier()
    t0 = time.perf_counter()
    tl.clear()
    run(warm, timed)
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
    out = {"value": round(aggregate_mpix(w, h, timed, world, el), 3), "unit": "Mpix/s",
           "ms_per_frame": round(el * 1e3 / timed, 4), "timed_frames": timed, "entropy_threads": a.entropy_threads,
           "staging_slots": stages, "pipeline": pipeline}
    if 0 < batch < timed and len(T) == timed:
        # between the first launch's last frame collected and the last frame
        # collected: no pipeline fill and no entropy tail of the last launch
        st_us = float(T[-1, 4] - T[batch - 1, 4])
        if st_us > 0:
            out["steady_value"] = round(w * h * (timed - batch) * world / st_us, 3)
    out["note"] = ("hot path + host entropy (native frame pipeline, cairo_stream_*); payload bits produced; "
                   "twice the timed leg's frames, every one a distinct resident frame of the same stream; each payload kept for the check")
    return out


def host_rgb(cairo_amd, a, w, h, ring, q, batch, local):
    """The hot path fed from host memory (PCIe-inclusive): frames in pinned
    host buffers, each uploaded by the context inside the timed region
    (cairo_ctx_submit with rgb_on_device = 0), feed outputs as in the timed
    leg.  Not the headline value (that has the frames resident in HBM)."""
    import torch

    steps = max(1, a.host_rgb_steps)
    warm, timed = batch, steps * batch
    # two launches' worth of distinct pinned frames, cycled: frame f is
    # host[f % n] (its references f-1..f-3 still differ), so the leg runs long
    # enough to amortise the first launch's uploads and the last launch's tail
    n = 2 * batch
    try:
        pinned = torch.empty((n, h, w, 3), dtype=torch.uint8, pin_memory=True)
    except RuntimeError as ex:  # pinned memory refused: report, do not fail the line
        return {"error": f"pinned host frames: {ex}"[:200]}
    host = pinned.numpy()
    with ThreadPoolExecutor(max(1, min(8, host_cpus()))) as pool:
        list(pool.map(lambda f: host.__setitem__(f, cairo_amd.make_band4(w, h, f)), range(n)))
    done = []  # completion time of every timed frame
    ctx = cairo_amd.Context(w, h, ring, device=local)
    ctx.set_batch(batch)
    ctx.set_outputs(cairo_amd.OUT_FEED)
    stages = ctx.stages

    def run(first, count, log=None):
        inflight = deque()

        def retire():
            ff, t = inflight.popleft()
            ctx.wait(t, copy=False)
            ctx.release(t)
            if log is not None:
                log.append(time.perf_counter())

        for f in range(first, first + count):
            if len(inflight) == stages:
                retire()
            inflight.append((f, ctx.submit(host[f % n], f, f > 0, q, on_device=False)))
        while inflight:
            retire()

    run(0, warm)
    ctx.sync()
    t0 = time.perf_counter()
    run(warm, timed, done)
    ctx.sync()
    el = time.perf_counter() - t0
    ctx.close()
    del host, pinned
    out = {"value": round(w * h * timed / el / 1e6, 3), "unit": "Mpix/s", "ms_per_frame": round(el * 1e3 / timed, 4),
           "timed_frames": timed, "pcie_bytes_per_frame": 3 * w * h,
           "pcie_GBps": round(3 * w * h * timed / el / 1e9, 2)}
    if timed > batch and len(done) == timed:
        # between the first launch's last frame and the last frame: no pipeline
        # fill (the first batch's uploads) and no unoverlapped last-launch tail
        # counted against the rate (launches overlap, each spans ~2 periods)
        st = done[-1] - done[batch - 1]
        out["steady_value"] = round(w * h * (timed - batch) / st / 1e6, 3)
        out["steady_ms_per_frame"] = round(st * 1e3 / (timed - batch), 4)
        out["steady_pcie_GBps"] = round(3 * w * h * (timed - batch) / st / 1e9, 2)
    out["note"] = ("frames in pinned host memory (2 launches' worth, cycled), uploaded per launch inside the timed "
                   "region (rgb_on_device=0); feed outputs; PCIe-inclusive rate, not the headline value")
    return out


def api_encode(w, h, ring, q, frames):
    """evx1_encoder::encode() timed by a C++ caller built against
    include/evx1.h (cairo_amd/_lib/evx1_api_caller): one synchronous call per
    frame, host RGB in, the stream appended to a bit_stream -- the
    reference's interface (evx1enc.cpp:92-156), PCIe and host entropy
    included."""
    if not os.path.exists(API_BIN):
        return {"error": f"{os.path.relpath(API_BIN, ROOT)} not built"}
    r = subprocess.run([API_BIN, str(w), str(h), str(ring), str(q), str(frames)], capture_output=True, text=True,
                       timeout=300)
    if r.returncode != 0:
        return {"error": f"exit {r.returncode}: {r.stderr[-400:]}"}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    ms = d["encode_ms"][1:]  # P-frames
    return {"value": round(w * h * len(ms) / (sum(ms) * 1e-3) / 1e6, 3), "unit": "Mpix/s",
            "ms_per_p_frame": round(float(np.mean(ms)), 3), "ms_i_frame": round(d["encode_ms"][0], 3),
            "fps": round(1e3 / float(np.mean(ms)), 2), "frames": frames, "stream_fnv1a64": d["fnv1a64"],
            "note": "synchronous evx1_encoder::encode() per frame (drop-in C++ API, vtable call, host RGB, "
                    "host entropy on the calling thread)"}


def cpu_baseline(cairo_amd, content, w, h, ring, q, pframes, last, hot_h, e2e_h, golden, batch):
    """The oracle (plain-C restatement of the reference encoder, test
    infrastructure) on one host core: frame 0 (I) + `pframes` P-frames timed
    (a bounded sample); P-frame Mpix/s.  It then continues, untimed, to frame
    `last`; the records of frames 0..last are hashed as the golden file's and
    compared with the GPU's (timed context, end-to-end pipeline) and with the
    golden file's prefix (the checker role) -> (baseline, sample check)."""
    from oracle import oracle as orc

    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    ref = []
    tp = 0.0
    orc.op_counts(reset=True)
    for t in range(last + 1):
        rgb = content_frame(content, w, h, t)
        t0 = time.perf_counter()
        data, n = e.encode(rgb)
        dt = time.perf_counter() - t0
        if 0 < t <= pframes:
            tp += dt
        ref.append(f"{orc.fnv1a64(orc.canonical_frame_bytes(data, n, t == 0)):016x}")
    base = {"value": round(w * h * pframes / tp / 1e6, 4), "unit": "Mpix/s", "cores": 1, "kind": "port",
            "sample": f"{w}x{h} q={q} R={ring}: frame 0 (I, untimed) + {pframes} P-frames timed, {content} content, "
                      f"oracle/evx_oracle.c -O3 -march=x86-64-v3, one thread",
            "cpu": cpu_model(), "host_cpus_available": host_cpus()}
    frames = range(last + 1)
    mism = sorted({t for t in frames if hot_h.get(t) != ref[t]} |
                  ({t for t in frames if e2e_h.get(t) != ref[t]} if e2e_h else set()))
    sample = {"frames": last + 1, "launches_covered": -(-(last + 1) // batch), "mismatched_frames": mism}
    if golden:
        have = golden["frame_fnv1a64"]
        sample["golden_prefix_matches"] = all(t < len(have) and have[t] == ref[t] for t in frames)
        if not sample["golden_prefix_matches"]:
            sample["mismatched_frames"] = sorted(set(mism) | {-1})  # -1: the golden file itself
    return base, sample


if __name__ == "__main__":
    main()
