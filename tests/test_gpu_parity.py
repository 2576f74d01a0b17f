"""GPU parity: the HIP encode path (libcairo_amd.so) against the oracle.

Bit-exact on every intermediate the reference exposes: the transform /
quantize / reconstruct chain on random macroblocks (KAT), and per frame the
inter-search records, the block table, the quantized coefficients
(output_cache), the reconstruction before and after the deblocking filter,
and finally whole streams through the drop-in evx1_encoder API against the
frozen stream hashes in tests/golden/oracle_streams.json (themselves pinned
to the reference's recorded sizes, tests/test_oracle.py).
"""
import json
import struct
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ---------------------------------------------------------------------------
# KAT: transform -> VAQ -> quantize -> dequantize -> inverse transform (+pred)
# ---------------------------------------------------------------------------

def _luma16(blocks):
    """block-major (6, 8, 8) -> 16x16 luma of quadrants TL TR BL BR."""
    y = np.empty((16, 16), np.int16)
    for b in range(4):
        y[(b >> 1) * 8:(b >> 1) * 8 + 8, (b & 1) * 8:(b & 1) * 8 + 8] = blocks[b]
    return y


def _blocks(y16, u, v):
    out = np.empty((6, 8, 8), np.int16)
    for b in range(4):
        out[b] = y16[(b >> 1) * 8:(b >> 1) * 8 + 8, (b & 1) * 8:(b & 1) * 8 + 8]
    out[4], out[5] = u, v
    return out


def _oracle_chain(orc, src, pred, typ, quality):
    L = orc.lib()
    P = lambda a: a.ctypes.data  # noqa: E731
    coef = np.zeros((6, 8, 8), np.int16)
    for b in range(6):
        s = np.ascontiguousarray(src[b])
        if typ == 1:
            L.orc_transform_8x8(P(s), 8, P(coef[b]), 8)
        else:
            p = np.ascontiguousarray(pred[b])
            L.orc_sub_transform_8x8(P(s), 8, P(p), 8, P(coef[b]), 8)
    y16 = _luma16(coef)
    q = L.orc_vaq(quality, P(y16), 16)
    var = L.orc_variance2(P(y16), 16)
    qy, qu, qv = np.zeros((16, 16), np.int16), np.zeros((8, 8), np.int16), np.zeros((8, 8), np.int16)
    u, v = np.ascontiguousarray(coef[4]), np.ascontiguousarray(coef[5])
    L.orc_quantize_mb(q, typ, P(y16), P(u), P(v), P(qy), P(qu), P(qv))
    dy, du, dv = np.zeros_like(qy), np.zeros_like(qu), np.zeros_like(qv)
    L.orc_dequantize_mb(q, typ, P(qy), P(qu), P(qv), P(dy), P(du), P(dv))
    deq = _blocks(dy, du, dv)
    rec = np.zeros((6, 8, 8), np.int16)
    for b in range(6):
        d = np.ascontiguousarray(deq[b])
        if typ == 1:
            L.orc_inverse_transform_8x8(P(d), 8, P(rec[b]), 8)
        else:
            p = np.ascontiguousarray(pred[b])
            L.orc_inverse_transform_add_8x8(P(d), 8, P(p), 8, P(rec[b]), 8)
    return _blocks(qy, qu, qv), rec, q, var


def test_kat_transform_chain(orc, cairo):
    rng = np.random.default_rng(2024)
    n = 96
    src = rng.integers(16, 272, (n, 6, 8, 8)).astype(np.int16)
    pred = rng.integers(-200, 600, (n, 6, 8, 8)).astype(np.int16)
    # edge content: flat, extreme, checkerboard
    src[0] = 16
    src[1] = 271
    pred[2] = -32000
    src[3] = np.where((np.indices((6, 8, 8)).sum(0) % 2) == 0, 16, 271)
    types = np.array([1, 0, 2, 3] * (n // 4), np.uint8)
    quals = np.array([1, 4, 8, 16, 24, 31] * (n // 6), np.uint8)
    qtype = np.stack([types, quals], 1).astype(np.uint8).copy()
    coef = np.zeros((n, 6, 8, 8), np.int16)
    rec = np.zeros_like(coef)
    qv = np.zeros((n, 2), np.int32)
    P = lambda a: a.ctypes.data  # noqa: E731
    st = cairo.lib().cairo_kat_transform(P(src), P(pred), P(qtype), n, P(coef), P(rec), P(qv), 0)
    assert st == 0
    for m in range(n):
        c, r, q, var = _oracle_chain(orc, src[m], pred[m], int(types[m]), int(quals[m]))
        assert qv[m, 0] == q, m
        assert qv[m, 1] == var, m
        np.testing.assert_array_equal(coef[m], c, err_msg=f"coef mb {m}")
        np.testing.assert_array_equal(rec[m], r, err_msg=f"recon mb {m}")


# ---------------------------------------------------------------------------
# Frame-level parity
# ---------------------------------------------------------------------------

def _table_equal(a, b, what):
    for f in a.dtype.names:
        if f == "pad":
            continue
        bad = np.nonzero(a[f] != b[f])[0]
        assert bad.size == 0, f"{what}: field {f} differs at MBs {bad[:10]} gpu={a[f][bad[:5]]} ref={b[f][bad[:5]]}"


def _run_frames(orc, cairo, w, h, ring, q, frames, intra_only=False, check_inter=True, gen=None):
    gen = gen or orc.make_frame
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    ctx = cairo.Context(w, h, ring)
    ctx.set_debug(1)
    for t in range(frames):
        rgb = gen(w, h, t)
        inter = t > 0 and not intra_only
        if intra_only:
            e.insert_intra()
        e.encode(rgb)
        out = ctx.encode_frame(rgb, t, inter, q)
        tag = f"{w}x{h} R={ring} q={q} frame {t}"
        gy, gu, gv = ctx.read_planes(0)
        oy, ou, ov = e.planes(0)
        np.testing.assert_array_equal(gy, oy, err_msg=f"{tag}: input Y")
        np.testing.assert_array_equal(gu, ou, err_msg=f"{tag}: input U")
        if inter and check_inter and ring > 1:
            gd, gs = ctx.read_inter()
            od, os_ = e.inter_records()
            _table_equal(gd, od, f"{tag}: inter records")
            np.testing.assert_array_equal(gs, os_, err_msg=f"{tag}: inter SAD")
        _table_equal(out.table, e.block_table(), f"{tag}: block table")
        oy, ou, ov = e.planes(1)
        np.testing.assert_array_equal(out.coef_y, oy, err_msg=f"{tag}: coef Y")
        np.testing.assert_array_equal(out.coef_u, ou, err_msg=f"{tag}: coef U")
        np.testing.assert_array_equal(out.coef_v, ov, err_msg=f"{tag}: coef V")
        py, pu, pv = ctx.read_predeblock()
        ry, ru, rv = e.predeblock()
        np.testing.assert_array_equal(py, ry, err_msg=f"{tag}: recon Y (pre-deblock)")
        np.testing.assert_array_equal(pu, ru, err_msg=f"{tag}: recon U (pre-deblock)")
        np.testing.assert_array_equal(pv, rv, err_msg=f"{tag}: recon V (pre-deblock)")
        slot = 2 + t % ring
        gy, gu, gv = ctx.read_planes(slot)
        oy, ou, ov = e.planes(slot)
        np.testing.assert_array_equal(gy, oy, err_msg=f"{tag}: recon Y (deblocked)")
        np.testing.assert_array_equal(gu, ou, err_msg=f"{tag}: recon U (deblocked)")
        np.testing.assert_array_equal(gv, ov, err_msg=f"{tag}: recon V (deblocked)")
    ctx.close()


@pytest.mark.parametrize("ring,q", [(4, 16), (2, 16), (4, 1), (4, 31), (3, 8)])
def test_frames_cif(orc, cairo, ring, q):
    _run_frames(orc, cairo, 352, 288, ring, q, 6)


def test_frames_cif_intra_only(orc, cairo):
    _run_frames(orc, cairo, 352, 288, 4, 16, 6, intra_only=True)


def test_frames_odd_sizes(orc, cairo):
    _run_frames(orc, cairo, 200, 120, 3, 16, 5)   # ragged MB grid, Wa > W
    _run_frames(orc, cairo, 64, 48, 2, 8, 4)      # tiny: 4x3 MBs
    _run_frames(orc, cairo, 16, 16, 2, 16, 3)     # one macroblock


def test_frames_720p(orc, cairo):
    _run_frames(orc, cairo, 1280, 720, 2, 16, 3)


def test_frames_1080p_padding(orc, cairo):
    _run_frames(orc, cairo, 1920, 1080, 4, 8, 2)  # Ha = 1088: 8 zero rows


def test_frames_4k(orc, cairo):
    """BASELINE.json configs[3] geometry (the largest frame): I + P, R = 4,
    every intermediate bit-exact."""
    _run_frames(orc, cairo, 3840, 2160, 4, 16, 2)


# Content beyond band4 (tests/content.py): noise, static, flat extremes,
# near-ties, out-of-range motion with a scene cut, sub-pel gradients.
@pytest.mark.parametrize("kind,q", [("noise", 16), ("static", 16), ("black", 8), ("white", 31), ("ties", 1), ("ties", 16),
                                    ("pan", 16), ("gradient", 1), ("gradient", 16)])
def test_frames_content(orc, cairo, kind, q):
    from tests import content

    _run_frames(orc, cairo, 352, 288, 4, q, 5, gen=lambda w, h, t: content.make(kind, w, h, t))


@pytest.mark.parametrize("kind", ["noise", "ties", "pan", "static"])
def test_batched_content(orc, cairo, kind):
    from tests import content

    _run_batched(orc, cairo, 352, 288, 2, 16, 12, 6, gen=lambda w, h, t: content.make(kind, w, h, t))


# ---------------------------------------------------------------------------
# Whole streams through the drop-in encoder (evx1_encoder API)
# ---------------------------------------------------------------------------

STREAMS = json.load(open(os.path.join(GOLD, "oracle_streams.json")))["configs"]


@pytest.mark.parametrize("cfg", STREAMS, ids=[c["name"] for c in STREAMS])
def test_encoder_stream_matches_golden(orc, cairo, cfg):
    enc = cairo.Encoder(ring=cfg["ring"])
    enc.set_quality(cfg["quality"])
    w, h = cfg["width"], cfg["height"]
    bs = cairo.BitStream(w * h * 64 + 65536)
    hsh = orc.FNV_OFFSET
    for t in range(cfg["frames"]):
        if cfg["intra_only"]:
            enc.insert_intra()
        bs.empty()
        enc.encode(cairo.make_band4(w, h, t), bs)
        n = bs.bits()
        assert n == cfg["frame_bits"][t], f"frame {t}"
        hsh = orc.fnv1a64(orc.canonical_frame_bytes(bs.data(), n, t == 0), hsh)
    assert f"{hsh:016x}" == cfg["fnv1a64"]
    enc.close()


# ---------------------------------------------------------------------------
# Pipelined batches: several frames in one engine launch (frames overlap on
# the GPU with row-level dependencies); every frame must still match.
# ---------------------------------------------------------------------------

def _payload_bits(cairo, out, ctx, ring, tk):
    """A frame's ABAC payload (after the header and frame descriptor) from its
    outputs, as a bit array: from the GPU precode's feed when valid, else from
    the planes (fetched for a feed-only context)."""
    if out.feed_status == cairo.FEED_VALID:
        data, n = cairo.serialize_feed(out.feed, out.feed_bits)
    else:
        cy, cu, cv = (out.coef_y, out.coef_u, out.coef_v) if out.coef_y is not None else ctx.fetch_coef(tk)
        data, n = cairo.serialize_slice(out.table, ctx.wmb, ctx.hmb, ring, cy, cu, cv)
    return np.unpackbits(np.frombuffer(data, np.uint8), bitorder="little")[:n]


class _DeviceFrames:
    """Frames uploaded to HBM before the run (as bench.py keeps them), through
    the HIP runtime the library itself uses; submitted by device address."""

    def __init__(self, frames):
        import ctypes

        self.hip = ctypes.CDLL("libamdhip64.so.7")  # by soname: the copy already loaded into this process
        self.n, self.size = len(frames), frames[0].nbytes
        self.ptr = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(self.ptr), ctypes.c_size_t(self.n * self.size)) == 0
        for t, f in enumerate(frames):
            assert self.hip.hipMemcpy(ctypes.c_void_p(self.ptr.value + t * self.size),
                                      f.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(self.size), 1) == 0

    def __getitem__(self, t):
        return self.ptr.value + t * self.size

    def free(self):
        if self.ptr.value:
            self.hip.hipFree(self.ptr)
            self.ptr.value = None


def _run_batched(orc, cairo, w, h, ring, q, frames, batch, intra_every=0, gen=None, workgroups=0, outputs=0,
                 device_frames=False):
    """Frames through one pipelined Context (up to `stages` in flight, `batch`
    frames per launch, 0 = the library default; consecutive launches overlap
    on two streams) vs the oracle: block table and coefficients of every
    frame, then every ring slot at the end.  outputs = the context's
    set_outputs (0: the default, coefficient planes); with OUT_FEED, as
    bench.py times it, every frame's payload bits (coded from the GPU
    precode's feed) are compared with the oracle's stream record too, and
    the coefficients are fetched from the staging slot.  device_frames: the
    frames are resident in HBM before the first submit and submitted by
    device address, as bench.py's timed region does."""
    gen = gen or orc.make_frame
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    ref = []
    for t in range(frames):
        rgb = gen(w, h, t)
        intra = t == 0 or (intra_every and t % intra_every == 0)
        if intra:
            e.insert_intra()
        data, nbits = e.encode(rgb)
        head = (14 * 8 if t == 0 else 0) + 10 * 8  # header + frame descriptor precede the payload
        bits = np.unpackbits(np.frombuffer(data, np.uint8), bitorder="little")[head:nbits]
        ref.append((intra, e.block_table(), e.planes(1), bits))
    final_slots = [e.planes(2 + k) for k in range(ring)]
    dev = _DeviceFrames([gen(w, h, t) for t in range(frames)]) if device_frames else None
    ctx = cairo.Context(w, h, ring)
    if outputs:
        ctx.set_outputs(outputs)
    if batch:
        ctx.set_batch(batch)
    if workgroups:
        ctx.set_workgroups(workgroups)
    stages = ctx.stages
    pending = []

    def check(t, tk):
        out = ctx.wait(tk)
        tag = f"{w}x{h} R={ring} q={q} batch={batch} frame {t}"
        _table_equal(out.table, ref[t][1], f"{tag}: block table")
        coef = (out.coef_y, out.coef_u, out.coef_v) if out.coef_y is not None else ctx.fetch_coef(tk)
        np.testing.assert_array_equal(coef[0], ref[t][2][0], err_msg=f"{tag}: coef Y")
        np.testing.assert_array_equal(coef[1], ref[t][2][1], err_msg=f"{tag}: coef U")
        np.testing.assert_array_equal(coef[2], ref[t][2][2], err_msg=f"{tag}: coef V")
        if outputs & cairo.OUT_FEED:
            assert out.feed_status == cairo.FEED_VALID, f"{tag}: feed status {out.feed_status}"
            got = _payload_bits(cairo, out, ctx, ring, tk)
            assert got.size == ref[t][3].size, f"{tag}: payload {got.size} vs {ref[t][3].size} bits"
            assert np.array_equal(got, ref[t][3]), f"{tag}: payload bits differ"
        ctx.release(tk)

    for t in range(frames):  # at most `stages` frames in flight (submitted, not released)
        if len(pending) == stages:
            check(*pending.pop(0))
        if dev is not None:
            pending.append((t, ctx.submit(dev[t], t, not ref[t][0], q, on_device=True)))
        else:
            pending.append((t, ctx.submit(gen(w, h, t), t, not ref[t][0], q)))
    for p in pending:
        check(*p)
    ctx.sync()
    for k in range(ring):
        gy, gu, gv = ctx.read_planes(2 + k)
        np.testing.assert_array_equal(gy, final_slots[k][0], err_msg=f"slot {k} Y")
        np.testing.assert_array_equal(gu, final_slots[k][1], err_msg=f"slot {k} U")
        np.testing.assert_array_equal(gv, final_slots[k][2], err_msg=f"slot {k} V")
    ctx.close()
    if dev is not None:
        dev.free()


@pytest.mark.parametrize("ring,batch", [(2, 8), (4, 8), (3, 5), (2, 1)])
def test_batched_cif(orc, cairo, ring, batch):
    _run_batched(orc, cairo, 352, 288, ring, 16, 12, batch)


def test_batched_mixed_intra(orc, cairo):
    _run_batched(orc, cairo, 352, 288, 4, 8, 12, 8, intra_every=3)


def test_batched_720p(orc, cairo):
    _run_batched(orc, cairo, 1280, 720, 2, 16, 10, 8)


def test_batched_ragged(orc, cairo):
    _run_batched(orc, cairo, 200, 120, 3, 16, 9, 4)
    _run_batched(orc, cairo, 16, 16, 2, 16, 6, 6)


@pytest.mark.parametrize("batch", [1, 3, 16])
def test_overlapping_launches_long(orc, cairo, batch):
    """Many launches in flight (consecutive launches overlap on two streams):
    40 CIF frames, R=2, an intra frame every 11th."""
    _run_batched(orc, cairo, 352, 288, 2, 16, 40, batch, intra_every=11)


def test_overlapping_launches_720p(orc, cairo):
    _run_batched(orc, cairo, 1280, 720, 2, 16, 20, 4)


# ---------------------------------------------------------------------------
# Frame pipeline (cairo_stream_*): GPU hot path + native entropy workers.
# Frame records assembled from its payloads must reproduce the reference
# stream (evx1enc.cpp:119-168 order: [header], frame desc, payload).
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("cfg", STREAMS, ids=[c["name"] for c in STREAMS])
def test_stream_matches_golden(orc, cairo, cfg):
    w, h, ring, q = cfg["width"], cfg["height"], cfg["ring"], cfg["quality"]
    ctx = cairo.Context(w, h, ring)
    ctx.set_batch(4)
    st = cairo.Stream(ctx, threads=3)
    frames = [cairo.make_band4(w, h, t) for t in range(cfg["frames"])]
    tks = [st.submit(f, t, not (cfg["intra_only"] or t == 0), q) for t, f in enumerate(frames)]
    hsh = orc.FNV_OFFSET
    for t, tk in enumerate(tks):
        typ = 0 if (cfg["intra_only"] or t == 0) else 1
        hdr = struct.pack("<4sHBxHHH", b"EVX1", 14, ring, (2 << 8) | 47, w, h) if t == 0 else b""
        head = hdr + struct.pack("<IIH", typ, t, q)
        buf = np.zeros(len(head) + w * h * 8, np.uint8)
        buf[: len(head)] = np.frombuffer(head, np.uint8)
        n = st.collect(tk, buf, len(head) * 8)
        assert n == cfg["frame_bits"][t], f"frame {t}"
        hsh = orc.fnv1a64(orc.canonical_frame_bytes(buf.tobytes(), n, t == 0), hsh)
    assert f"{hsh:016x}" == cfg["fnv1a64"]
    st.close()
    ctx.close()


def test_stream_long_unaligned(orc, cairo):
    """90 CIF frames (more than 2 x stages in flight over time), R=2, intra
    every 11th, payloads appended back to back at unaligned bit offsets into
    one buffer; every frame record equals the oracle encoder's."""
    w, h, ring, q, n = 352, 288, 2, 16, 90
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    ctx = cairo.Context(w, h, ring)
    st = cairo.Stream(ctx, threads=4)
    stages = ctx.L.cairo_ctx_stages(ctx.h)
    out = np.zeros(n * w * h, np.uint8)
    pos = 0
    inflight = []
    ref = []
    for t in range(n):
        intra = t % 11 == 0
        if intra:
            e.insert_intra()
        rgb = orc.make_frame(w, h, t)
        data, nb = e.encode(rgb)
        ref.append((data, nb, intra))
        if len(inflight) == stages:
            tt, tk = inflight.pop(0)
            pos = _append_record(st, out, pos, tt, tk, ref, w, h, ring, q)
        inflight.append((t, st.submit(rgb, t, not intra, q)))
    for tt, tk in inflight:
        pos = _append_record(st, out, pos, tt, tk, ref, w, h, ring, q)
    # the concatenated records, frame by frame
    p = 0
    for t, (data, nb, _) in enumerate(ref):
        want = np.unpackbits(np.frombuffer(data, np.uint8), bitorder="little")[:nb]
        got = np.unpackbits(out, bitorder="little")[p:p + nb]
        if t == 0:  # header pad byte 7
            want = want.copy()
            got = got.copy()
            want[56:64] = 0
            got[56:64] = 0
        np.testing.assert_array_equal(got, want, err_msg=f"frame {t}")
        p += nb
    assert p == pos
    st.close()
    ctx.close()


def _append_record(st, out, pos, t, tk, ref, w, h, ring, q):
    intra = ref[t][2]
    hdr = struct.pack("<4sHBxHHH", b"EVX1", 14, ring, (2 << 8) | 47, w, h) if t == 0 else b""
    head = hdr + struct.pack("<IIH", 0 if intra else 1, t, q)
    import cairo_amd

    pos = cairo_amd.bits_append(out, pos, head, len(head) * 8)
    return st.collect(tk, out, pos)


# ---------------------------------------------------------------------------
# The drop-in decoder (evx1_decoder): host entropy decode + the decode-mode
# engine + convert_image.  Decoding the encoder's stream must give exactly the
# encoder's reconstruction (the reference is closed-loop: decoder output ==
# peek(DESTINATION)), i.e. the oracle's deblocked ring slot,
# converted to RGB.
# ---------------------------------------------------------------------------

def _decode_round_trip(orc, cairo, w, h, ring, q, frames, intra_every=0):
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    enc = cairo.Encoder(ring=ring)
    enc.set_quality(q)
    dec = cairo.Decoder()
    bs = cairo.BitStream(w * h * 64 + 65536)
    for t in range(frames):
        if intra_every and t % intra_every == 0:
            e.insert_intra()
            enc.insert_intra()
        rgb = orc.make_frame(w, h, t)
        e.encode(rgb)
        bs.empty()
        enc.encode(rgb, bs)
        out = dec.decode(bs, w, h)
        assert bs.bits() == 0  # decode empties its input (evx1dec.cpp:121)
        want = cairo.yuv_to_rgb(*e.planes(2 + t % ring), w, h)
        np.testing.assert_array_equal(out, want, err_msg=f"{w}x{h} R={ring} q={q} frame {t}")
    dec.close()
    enc.close()


@pytest.mark.parametrize("ring,q", [(4, 16), (2, 16), (4, 1), (4, 31)])
def test_decoder_cif(orc, cairo, ring, q):
    _decode_round_trip(orc, cairo, 352, 288, ring, q, 8)


def test_decoder_intra_and_ragged(orc, cairo):
    _decode_round_trip(orc, cairo, 352, 288, 4, 8, 9, intra_every=4)
    # (R = 3 does not round-trip in the reference either: prediction targets
    # are written with log2(R) = 1 bit, serialize.cpp:179, so target 2 reads as 0)
    _decode_round_trip(orc, cairo, 200, 120, 2, 16, 6)
    _decode_round_trip(orc, cairo, 64, 48, 4, 16, 5)


def test_decoder_720p(orc, cairo):
    _decode_round_trip(orc, cairo, 1280, 720, 2, 16, 4)


def test_decoder_4k(orc, cairo):
    _decode_round_trip(orc, cairo, 3840, 2160, 4, 16, 3)


def test_decoder_rejects_bad_streams(cairo):
    dec = cairo.Decoder()
    bs = cairo.BitStream(4096)
    bs.write(b"XVX1" + bytes(20))
    with pytest.raises(cairo.CairoError):
        dec.decode(bs, 64, 48)
    dec.close()
