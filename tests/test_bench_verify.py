"""bench.py's every-frame check on CPU: the host store the timed region
copies feeds into, the record hashing, and the golden stream files
(tests/golden/stream_*.json, made by make_stream_golden.py) against the
oracle's live records."""
import json
import os

import numpy as np
import pytest

import bench

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_arena_reserve_and_grow():
    a = bench.Arena(chunk=1 << 12)
    a.grow(3 << 12)
    n0 = len(a.chunks)
    assert n0 == 3
    seen = []
    for k in range(20):
        buf, off = a.reserve(500)
        assert off % 16 == 0 and off + 500 <= buf.size
        buf[off:off + 500] = k
        seen.append((buf, off, k))
    assert len(a.chunks) == n0  # 20 x 512 bytes fit the pre-touched chunks: no allocation
    for buf, off, k in seen:  # nothing overwritten
        assert (buf[off:off + 500] == k).all()
    buf, off = a.reserve(1 << 14)  # larger than a chunk: one of its own
    assert buf.size >= 1 << 14 and off == 0


def _payload(data, nbits, t):
    """The payload of an oracle frame record: bits after the header (frame 0)
    and the 10-byte frame descriptor, re-packed LSB-first from bit 0."""
    head = (14 * 8 if t == 0 else 0) + 10 * 8
    bits = np.unpackbits(np.frombuffer(data, np.uint8), bitorder="little")[head:nbits]
    return np.packbits(bits, bitorder="little").tobytes(), bits.size


def test_frame_hashes_match_golden_hashing(orc, cairo):
    """Payloads kept in a FrameStore (either kind) hash to exactly what
    make_stream_golden.py writes for the oracle's own records."""
    w, h, ring, q, n = 352, 288, 4, 16, 6
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    store = bench.FrameStore()
    want = {}
    for t in range(n):
        data, nb = e.encode(cairo.make_band4(w, h, t))
        want[t] = f"{orc.fnv1a64(orc.canonical_frame_bytes(data, nb, t == 0)):016x}"
        pay, pbits = _payload(data, nb, t)
        if t % 2:
            store.items[t] = ("bytes", pay, pbits)
        else:
            buf, off = store.arena.reserve(len(pay) + 8)
            buf[off:off + len(pay)] = np.frombuffer(pay, np.uint8)
            store.items[t] = ("pay", buf, off, pbits)
    got = bench.frame_hashes(cairo, store, w, h, ring, q, threads=3)
    assert got == want
    gold = {"frame_fnv1a64": [want[t] for t in range(n - 1)]}
    r = bench.check_hashes(got, gold, range(n), 2)
    assert (r["frames_checked"], r["timed_frames_checked"], r["unchecked_frames"], r["mismatches"]) == (5, 3, 1, 0)
    got[3] = "0" * 16
    assert bench.check_hashes(got, gold, range(n), 2)["mismatched_frames"] == [3]


def _golden_files():
    return sorted(f for f in os.listdir(GOLD) if f.startswith("stream_") and f.endswith(".json"))


@pytest.mark.parametrize("name", _golden_files())
def test_golden_stream_file_matches_oracle(orc, name):
    """Each committed golden stream: complete, one hash per frame, and its
    first frames re-made by the oracle here."""
    g = json.load(open(os.path.join(GOLD, name)))
    assert g["complete"] and g["frames"] == len(g["frame_fnv1a64"]) == len(g["frame_bits"])
    assert g["content"] in ("band4", "noise", "static")
    w, h, ring, q = g["width"], g["height"], g["ring"], g["quality"]
    assert bench.golden_stream(g["config"], g["content"], q, ring)["frames"] == g["frames"]
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    for t in range(2 if w * h > 2_000_000 else 4):
        data, nb = e.encode(bench.content_frame(g["content"], w, h, t))
        assert nb == g["frame_bits"][t], t
        assert f"{orc.fnv1a64(orc.canonical_frame_bytes(data, nb, t == 0)):016x}" == g["frame_fnv1a64"][t], t


def test_bench_goldens_cover_the_default_run():
    """The default bench run (3 warm-up + 20 timed launches of 32 frames, and
    the end-to-end leg's twice as many timed frames) is covered by the 4K
    golden, so every timed frame is checked."""
    g = bench.golden_stream("4k", "band4", 16, 4)
    assert g is not None and g["complete"]
    assert g["frames"] >= 3 * 32 + 2 * 20 * 32
