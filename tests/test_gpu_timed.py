"""GPU parity of the configurations bench.py times, and of the drop-in API.

* The pipelined Context with the library's default frames per launch (32 at
  every bench size), several launches in flight on two streams sharing their
  worker pools and, above 4000 macroblocks, helper issue priority: exactly
  what bench.py's timed region runs (BASELINE.json configs[1..4]), frame by
  frame against the oracle (block table, coefficients) and every ring slot at
  the end; and over 160-200 frames (five or more launches, recycled sync
  areas) against the oracle's golden stream hashes.
* evx1_encoder::encode() called from C++ through the vtable
  (tests/api/evx1_api_caller.cpp, built against include/evx1.h), peek() views,
  periodic intra (evx1enc.cpp:143-150), recovery after a reported timeout, the
  synchronous encoder's memory footprint, and reduced worker pools.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from tests.test_gpu_parity import _run_batched, _table_equal

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
API_BIN = os.path.join(ROOT, "cairo_amd", "_lib", "evx1_api_caller")


# ---------------------------------------------------------------------------
# The timed configurations, library defaults
# ---------------------------------------------------------------------------

def test_timed_720p_default_batch(orc, cairo):
    """configs[1]: 720p q=16 R=2, default 32 frames per launch, 40 frames = a
    full launch + a partial one overlapping it; feed outputs as bench.py
    times them, every frame's payload bits against the oracle's record."""
    assert cairo.default_batch(1280, 720) == 32
    _run_batched(orc, cairo, 1280, 720, 2, 16, 40, 0, outputs=cairo.OUT_FEED)


def test_timed_1080p_default_batch(orc, cairo):
    """configs[2]: 1080p q=8 R=4 (8 zero rows of padding), default 32 frames
    per launch, 36 frames: all three references live, two overlapping
    launches; feed outputs, payloads checked."""
    assert cairo.default_batch(1920, 1080) == 32
    _run_batched(orc, cairo, 1920, 1080, 4, 8, 36, 0, outputs=cairo.OUT_FEED)


def test_timed_4k_default_batch(orc, cairo):
    """configs[3] on one GPU: 4K q=16 R=4, default 32 frames per launch with
    helper priority, 35 frames: two overlapping launches, 3 live references;
    feed outputs (bench.py's timed mode), payloads checked."""
    assert cairo.default_batch(3840, 2160) == 32
    _run_batched(orc, cairo, 3840, 2160, 4, 16, 35, 0, outputs=cairo.OUT_FEED)


def test_timed_4k_many_launches(orc, cairo):
    """configs[3] past the first launches: 4K q=16 R=4 with the bench's
    banded queues, helper priority, feed outputs and device-resident frames,
    10 frames per launch, 44 frames = 5 launches.  Launch b reuses the sync
    area and task queue of launch b-3 (backend.hip flush: areas rotate mod 3)
    while launch b-1 still runs beside it, so launches 3 and 4 run on
    recycled sync state (the frame views are a 64-slot ring, not recycled
    here: test_many_launches_queued covers that); every frame's payload bits,
    block table and coefficients and every ring slot at the end against the
    oracle."""
    _run_batched(orc, cairo, 3840, 2160, 4, 16, 44, 10, outputs=cairo.OUT_FEED, device_frames=True)


def test_carry_chain_4k_many_launches(cairo):
    """The round-5 red run's configuration (test_timed_4k_many_launches: 4K
    q=16 R=4, device frames, feed outputs, 10 frames per launch, 44 frames),
    repeated in one process with no oracle time: every copy macroblock's
    coefficients must equal the previous frame's at the same place (the
    output_cache carry, encode.cpp:69-163 leaves them untouched), the
    previous frame's plane itself being pinned through the golden stream
    (every frame's payload hash, whose DC prediction reads copy neighbours'
    carried coefficients, serialize.cpp:58-72).  DESIGN §2."""
    import ctypes

    import bench
    from oracle import oracle as orc

    w, h, ring, q = 3840, 2160, 4, 16
    frames, batch, iters = 44, 10, 3
    g = bench.golden_stream("4k", "band4", q, ring)
    wmb, hmb = w // 16, (h + 15) // 16
    hip = ctypes.CDLL("libamdhip64.so.7")
    size = w * h * 3
    dev = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(frames * size)) == 0
    try:
        for t in range(frames):
            f = cairo.make_band4(w, h, t)
            assert hip.hipMemcpy(ctypes.c_void_p(dev.value + t * size), f.ctypes.data_as(ctypes.c_void_p),
                                 ctypes.c_size_t(size), 1) == 0
        for it in range(iters):
            ctx = cairo.Context(w, h, ring)
            ctx.set_outputs(cairo.OUT_FEED)
            ctx.set_batch(batch)
            tks = [ctx.submit(dev.value + t * size, t, t > 0, q, on_device=True) for t in range(frames)]
            prev = None
            for t, tk in enumerate(tks):
                out = ctx.wait(tk)
                data, nb = bench.record(cairo, w, h, ring, q, t, *bench.payload(cairo, ctx, out, tk))
                got = f"{orc.fnv1a64(orc.canonical_frame_bytes(data, nb, t == 0)):016x}"
                assert got == g["frame_fnv1a64"][t], f"iteration {it} frame {t}: record differs from the golden"
                cy, cu, cv = (np.array(p, copy=True) for p in ctx.fetch_coef(tk))
                if prev is not None:
                    copy = ((out.table["block_type"] & 4) != 0).reshape(hmb, wmb)
                    diff = (cy[: hmb * 16].reshape(hmb, 16, wmb, 16) !=
                            prev[0][: hmb * 16].reshape(hmb, 16, wmb, 16)).any(axis=(1, 3))
                    for cp, pp in ((cu, prev[1]), (cv, prev[2])):
                        diff |= (cp[: hmb * 8].reshape(hmb, 8, wmb, 8) !=
                                 pp[: hmb * 8].reshape(hmb, 8, wmb, 8)).any(axis=(1, 3))
                    bad = np.argwhere(copy & diff)
                    assert bad.size == 0, \
                        f"iteration {it} frame {t}: copy MBs (row, col) {bad[:8].tolist()} lost the previous coefficients"
                prev = (cy, cu, cv)
                ctx.release(tk)
            ctx.sync()
            ctx.close()
    finally:
        hip.hipFree(dev)


def _golden_stream_run(cairo, config, frames, batch=0, content="band4", host=False):
    """bench.py's timed leg exactly (its run_hot_path, FrameStore and record
    hashing): `frames` frames of `content` (bench.content_frame) resident in HBM, the library's default
    frames per launch, feed outputs, up to `stages` in flight; every frame's
    record hash against tests/golden/stream_<config>_*.json (the oracle's, made
    off-box), so long runs need no oracle time here.  host: the frames stay in
    host memory and the context uploads each at submit (bench.py's host_rgb
    leg; with feed outputs only, the uploads share the copy stream and the
    feed copies run on the launch stream)."""
    import ctypes

    import bench

    w, h, ring, q, _ = bench.CONFIGS[config]
    g = bench.golden_stream(config, content, q, ring)
    assert g is not None and g["frames"] >= frames, f"golden stream for {config} has too few frames"
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime the library uses
    size = w * h * 3
    dev = ctypes.c_void_p()
    hostf = []
    if not host:
        assert hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(frames * size)) == 0
    try:
        for t in range(frames):
            f = bench.content_frame(content, w, h, t)
            if host:
                hostf.append(f)
            else:
                assert hip.hipMemcpy(ctypes.c_void_p(dev.value + t * size), f.ctypes.data_as(ctypes.c_void_p),
                                     ctypes.c_size_t(size), 1) == 0
        ctx = cairo.Context(w, h, ring)
        ctx.set_outputs(cairo.OUT_FEED)
        if batch:
            ctx.set_batch(batch)
        store = bench.FrameStore()
        bench.run_hot_path(ctx, (lambda t: hostf[t]) if host else (lambda t: dev.value + t * size), 0, frames, q,
                           ctx.stages, lambda t, out, tk: store.keep_feed(cairo, ctx, t, out, tk), on_device=not host)
        ctx.sync()
        ctx.close()
    finally:
        if not host:
            hip.hipFree(dev)
    got = bench.frame_hashes(cairo, store, w, h, ring, q, threads=8)
    r = bench.check_hashes(got, g, range(frames), 0)
    assert r["frames_checked"] == frames
    assert r["mismatches"] == 0, f"{config}: frames {r['mismatched_frames']} differ from the golden stream"


def test_timed_4k_golden_160(cairo):
    """configs[3] at the bench's default 32 frames per launch over 160
    frames: five launches, so launches 3 and 4 run on sync areas, task queues
    and queue counters recycled from launches 0 and 1 (areas rotate mod 3),
    every frame's payload against the oracle's golden hashes."""
    assert cairo.default_batch(3840, 2160) == 32
    _golden_stream_run(cairo, "4k", 160)


def test_timed_1080p_golden_160(cairo):
    """configs[2] (q=8, R=4), 160 frames at 32 per launch, against the golden stream."""
    _golden_stream_run(cairo, "1080p", 160)


def test_timed_720p_golden_200(cairo):
    """configs[1] (q=16, R=2), 200 frames at 32 per launch, against the golden stream."""
    _golden_stream_run(cairo, "720p", 200)


@pytest.mark.parametrize("config,frames", [("720p", 100), ("4k", 70)])
def test_timed_host_rgb_golden(cairo, config, frames):
    """The host-RGB path (frames uploaded by the context at submit, feed
    outputs only: the uploads on the copy stream, the feed copies on the launch
    stream), several launches of 32, every frame against the golden stream."""
    _golden_stream_run(cairo, config, frames, host=True)


@pytest.mark.parametrize("content", ["noise", "static"])
def test_timed_4k_content_golden_160(cairo, content):
    """SURVEY §8(d)'s stress content at the bench's configuration, 160
    frames (five launches of 32): noise (every macroblock searched and coded,
    no copy exits) and a static scene (copy chains: each macroblock's
    coefficients carried from the previous frame's output_cache, the case the
    coefficient drain before the info granule protects), against their
    golden streams."""
    _golden_stream_run(cairo, "4k", 160, content=content)


def test_timed_4k_both_outputs(orc, cairo):
    """The same launches with both outputs (coefficient planes D2H and the
    feed): 4K, 6 frames."""
    _run_batched(orc, cairo, 3840, 2160, 4, 16, 6, 0, outputs=cairo.OUT_FEED | cairo.OUT_COEF)


@pytest.mark.parametrize("q,frames", [(1, 35), (8, 35), (31, 35)])
def test_4k_quality_sweep(orc, cairo, q, frames):
    """configs[4]: the 4K quality sweep (VAQ on), default launch, feed
    outputs.  q = 1 and 31 (the ends of the sweep) and 8 over 35 frames: two
    overlapping launches (32 + 3 frames), every payload against the oracle."""
    _run_batched(orc, cairo, 3840, 2160, 4, q, frames, 0, outputs=cairo.OUT_FEED)


@pytest.mark.parametrize("rows", [1, 3])
def test_reduced_worker_pools(orc, cairo, rows):
    """One or three row coders / helpers per launch (a partly resident launch
    degenerates to this): the task queues still drain in dependency order."""
    _run_batched(orc, cairo, 352, 288, 4, 16, 10, 4, workgroups=rows)


def test_workgroup_cap(cairo):
    ctx = cairo.Context(352, 288, 2)
    with pytest.raises(cairo.CairoError):
        ctx.set_workgroups(100000)  # more than stays co-resident with the other launch
    ctx.close()


# ---------------------------------------------------------------------------
# The drop-in API
# ---------------------------------------------------------------------------

def _api(args):
    assert os.path.exists(API_BIN), "build with make (cairo_amd/_lib/evx1_api_caller)"
    r = subprocess.run([API_BIN] + [str(a) for a in args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_streams.json")))["configs"]


@pytest.mark.parametrize("cfg", [c for c in GOLD if not c["intra_only"]], ids=lambda c: c["name"])
def test_cpp_caller_matches_golden(cfg):
    """A C++ program built against include/evx1.h drives evx1_encoder through
    its vtable; its stream equals the frozen oracle stream."""
    d = _api([cfg["width"], cfg["height"], cfg["ring"], cfg["quality"], cfg["frames"]])
    assert d["frame_bits"] == cfg["frame_bits"]
    assert d["fnv1a64"] == cfg["fnv1a64"]


def test_cpp_caller_4k(orc, tmp_path):
    """The drop-in API at BASELINE configs[3] geometry: three frames."""
    w, h, ring, q, n = 3840, 2160, 4, 16, 3
    rec = tmp_path / "rec.bin"
    d = _api([w, h, ring, q, n, "--records", rec])
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    raw = rec.read_bytes()
    p = 0
    for t in range(n):
        nb = int(np.frombuffer(raw[p:p + 4], np.uint32)[0])
        got = raw[p + 4:p + 4 + (nb + 7) // 8]
        p += 4 + (nb + 7) // 8
        data, want_bits = e.encode(orc.make_frame(w, h, t))
        assert nb == want_bits == d["frame_bits"][t], t
        assert orc.canonical_frame_bytes(got, nb, t == 0) == orc.canonical_frame_bytes(data, nb, t == 0), t


def test_periodic_intra(orc, cairo):
    """evx1enc.cpp:143-150: after frame index 3599 ((index + 1) % 3600 == 0)
    the next frame is intra.  3603 frames of one macroblock through the
    drop-in encoder, every record against the oracle's."""
    w = h = 16
    enc = cairo.Encoder(ring=4)
    enc.set_quality(16)
    e = orc.OracleEncoder(4)
    e.set_quality(16)
    bs = cairo.BitStream(1 << 16)
    types = []
    for t in range(3603):
        rgb = orc.make_frame(w, h, t)
        bs.empty()
        enc.encode(rgb, bs)
        data, nb = e.encode(rgb)
        got = bs.data()
        assert bs.bits() == nb, t
        assert orc.canonical_frame_bytes(got, nb, t == 0) == orc.canonical_frame_bytes(data, nb, t == 0), t
        off = 14 if t == 0 else 0  # frame descriptor {type u32, index u32, quality u16}
        types.append(int(np.frombuffer(got[off:off + 4], np.uint32)[0]))
        assert int(np.frombuffer(got[off + 4:off + 8], np.uint32)[0]) == t
    assert types[0] == 0 and types[3600] == 0
    assert all(types[t] == 1 for t in range(1, 3603) if t != 3600)
    enc.close()


def _peek_views(orc, cairo, e, w, h, ring, index):
    """The reference's peek() views (evx1enc.cpp:170-305) from the oracle's state."""
    wmb = ((w + 15) // 16)
    tb = e.block_table()
    jj, ii = np.mgrid[0:h, 0:w]
    d = tb[(ii // 16) + (jj // 16) * wmb]
    copy = (d["block_type"] & 4) != 0
    out = {}
    v = np.zeros((h, w, 3), np.uint8)
    v[..., 2] = 255 * copy
    v[..., 1] = 255 * ((d["block_type"] & 2) != 0)
    v[..., 0] = 255 * ((d["block_type"] & 1) != 0)
    out[cairo.PEEK_BLOCK_TABLE] = v
    v = np.zeros((h, w, 3), np.uint8)
    qv = ((255 - 15 * d["q_index"].astype(np.int32)) & 255).astype(np.uint8)
    for c in range(3):
        v[..., c] = np.where(copy, 255 if c == 0 else 0, qv)
    out[cairo.PEEK_QUANT_TABLE] = v
    v = np.zeros((h, w, 3), np.uint8)
    var = np.clip(np.trunc(d["variance"].astype(np.int32) / 30), 0, 255).astype(np.uint8)
    for c in range(3):
        v[..., c] = np.where(copy, 255 if c == 0 else 0, var)
    out[cairo.PEEK_BLOCK_VARIANCE] = v
    v = np.zeros((h, w, 3), np.uint8)
    sp = d["sp_pred"] != 0
    v[..., 1] = np.where(sp, 255 * d["sp_amount"], 0)
    v[..., 2] = np.where(sp, 255 * (d["sp_amount"] == 0), 0)
    out[cairo.PEEK_SPMP_TABLE] = v
    out[cairo.PEEK_SOURCE] = cairo.yuv_to_rgb(*e.planes(0), w, h)
    out[cairo.PEEK_DESTINATION] = cairo.yuv_to_rgb(*e.planes(2 + index % ring), w, h)
    return out


def test_peek_views(orc, cairo):
    """peek() of every implemented state after each of 4 frames (I + 3 P),
    ragged size; PREDICTION is not implemented in the reference either."""
    w, h, ring, q = 200, 120, 4, 8
    enc = cairo.Encoder(ring=ring)
    enc.set_quality(q)
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    bs = cairo.BitStream(w * h * 64 + 65536)
    for t in range(4):
        rgb = orc.make_frame(w, h, t)
        bs.empty()
        enc.encode(rgb, bs)
        e.encode(rgb)
        for state, want in _peek_views(orc, cairo, e, w, h, ring, t).items():
            np.testing.assert_array_equal(enc.peek(state, w, h), want, err_msg=f"frame {t} peek state {state}")
        with pytest.raises(cairo.CairoError):
            enc.peek(cairo.PEEK_PREDICTION, w, h)
    enc.close()


def test_reset_recovers_after_timeout(orc, cairo):
    """A reported in-kernel timeout fails every frame until cairo_ctx_reset,
    which restores a fresh-encoder state (common.cpp:79-150): the next stream
    is bit-exact.  The report names the wait: first the host's mark (test
    hook 8), then a row helper's progress wait recorded by the device's own
    timeout path (test hook 16): kind, frame epoch and index, MB row,
    member, the awaited row, the columns it needed."""
    w, h, ring, q = 352, 288, 2, 16
    ctx = cairo.Context(w, h, ring)
    assert ctx.timeout_info() is None
    ctx.encode_frame(orc.make_frame(w, h, 0), 0, False, q)
    ctx.set_debug(8)
    with pytest.raises(cairo.CairoError) as ei:
        ctx.encode_frame(orc.make_frame(w, h, 1), 1, True, q)
    assert ei.value.status == cairo.EVX_ERROR_HARDWAREFAIL
    assert ei.value.timeout["kind"] == "host_mark"
    cairo.lib().cairo_ctx_reset(ctx.h)
    assert ctx.timeout_info() is None
    ctx.encode_frame(orc.make_frame(w, h, 0), 0, False, q)  # epoch 1
    ctx.set_debug(16)
    with pytest.raises(cairo.CairoError) as ei:
        ctx.encode_frame(orc.make_frame(w, h, 1), 1, True, q)  # epoch 2
    assert ei.value.status == cairo.EVX_ERROR_HARDWAREFAIL
    info = ctx.timeout_info()
    assert info == ei.value.timeout
    # row 1's helper, its first wait: frame index-2 is none yet at frame 1
    # (R = 2: no older reference), so the previous frame's progress of row
    # min(r + 2, hmb - 1) = 3 at the level-1 window of group 0 (80 columns)
    assert info["kind"] == "injected" and info["member"] == 0
    assert (info["epoch"], info["index"], info["row"]) == (2, 1, 1)
    assert (info["on"] & 0xFFFF, info["on"] >> 16, info["need"]) == (3, 1, 80)
    ctx.set_debug(0)
    cairo.lib().cairo_ctx_reset(ctx.h)
    assert ctx.timeout_info() is None
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    for t in range(3):
        rgb = orc.make_frame(w, h, t)
        e.encode(rgb)
        out = ctx.encode_frame(rgb, t, t > 0, q)
        _table_equal(out.table, e.block_table(), f"after reset, frame {t}")
        np.testing.assert_array_equal(out.coef_y, e.planes(1)[0])
    ctx.close()


def _hbm_free():
    """Free device memory through the HIP runtime the library itself uses
    (a second runtime, e.g. torch's bundled one, may not see the GPU once
    this one holds it)."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so.7")  # by soname: the copy already loaded into this process
    free, total = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
    return free.value


def test_sync_encoder_memory_4k(cairo):
    """The synchronous drop-in encoder keeps 2 staging slots: a 4K R=4
    instance takes well under 1 GB of HBM (64 slots would be about 8 GB)."""
    free0 = _hbm_free()
    enc = cairo.Encoder(ring=4)
    enc.set_quality(16)
    bs = cairo.BitStream(3840 * 2160 * 64)
    enc.encode(cairo.make_band4(3840, 2160, 0), bs)
    free1 = _hbm_free()
    enc.close()
    used = free0 - free1
    assert used < 1 << 30, f"{used / 2**20:.0f} MiB"


def test_submit_rejects_host_pointer_as_device(cairo):
    """rgb_on_device with a host address is refused before any kernel reads
    it (a device-side read of it would fault the GPU)."""
    w, h = 352, 288
    ctx = cairo.Context(w, h, 2)
    rgb = cairo.make_band4(w, h, 0)
    with pytest.raises(cairo.CairoError):
        ctx.submit(rgb.ctypes.data, 0, False, 16, on_device=True)
    out = ctx.encode_frame(rgb, 0, False, 16)  # the context is still usable
    assert out.table.size == ctx.wmb * ctx.hmb
    ctx.close()


def test_many_launches_queued(orc, cairo):
    """More launches queued than the context keeps frame-view slots for (64):
    96 staging slots, one frame per launch, 80 device frames submitted before
    the first wait.  Each view slot is rewritten only after its earlier copy
    to the device ran (backend.hip fdesc_done), so every frame is encoded from
    its own views."""
    import ctypes

    w, h, ring, q, n = 64, 48, 2, 16, 80
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime the library uses
    frames = np.stack([orc.make_frame(w, h, t) for t in range(n)])
    dev = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(frames.nbytes)) == 0
    try:
        assert hip.hipMemcpy(dev, frames.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(frames.nbytes), 1) == 0
        ctx = cairo.Context(w, h, ring)
        assert ctx.stages == 96
        ctx.set_batch(1)
        fsz = w * h * 3
        tks = [ctx.submit(dev.value + t * fsz, t, t > 0, q, on_device=True) for t in range(n)]
        e = orc.OracleEncoder(ring)
        e.set_quality(q)
        for t, tk in enumerate(tks):
            e.encode(frames[t])
            out = ctx.wait(tk)
            _table_equal(out.table, e.block_table(), f"frame {t}")
            np.testing.assert_array_equal(out.coef_y, e.planes(1)[0], err_msg=f"frame {t}")
            ctx.release(tk)
        ctx.close()
    finally:
        hip.hipFree(dev)


def test_host_rgb_release_without_wait(orc, cairo):
    """A caller may release a ticket without waiting for it (cairo_ctx_release
    needs no wait).  Host RGB frames are uploaded at submit into their staging
    slot's buffer, so a later frame's upload into the same slot must wait for
    the launch that converts the earlier frame (backend.hip rgb_read), or the
    earlier frame is encoded from the later image.  4 staging slots, 2 frames
    per launch, every ticket but the last released unwaited: the final ring
    slots and the last frame's outputs equal the oracle's."""
    w, h, ring, q, n = 352, 288, 4, 16, 14
    ctx = cairo.Context(w, h, ring, stages=4)
    ctx.set_batch(2)
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    tk = None
    for t in range(n):
        rgb = orc.make_frame(w, h, t)
        e.encode(rgb)
        tk = ctx.submit(rgb, t, t > 0, q)
        if t < n - 1:
            ctx.release(tk)
    out = ctx.wait(tk)
    _table_equal(out.table, e.block_table(), "last frame")
    np.testing.assert_array_equal(out.coef_y, e.planes(1)[0])
    ctx.release(tk)
    ctx.sync()
    for k in range(ring):
        gy, gu, gv = ctx.read_planes(2 + k)
        np.testing.assert_array_equal(gy, e.planes(2 + k)[0], err_msg=f"slot {k} Y")
        np.testing.assert_array_equal(gu, e.planes(2 + k)[1], err_msg=f"slot {k} U")
        np.testing.assert_array_equal(gv, e.planes(2 + k)[2], err_msg=f"slot {k} V")
    ctx.close()
