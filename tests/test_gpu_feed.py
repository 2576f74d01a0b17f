"""The GPU entropy precode (precode.hip): the feed bits
a frame hands to the host's arithmetic coder must make exactly the payload
the host precode makes from the block table and coefficients (and hence the
oracle's, tests/test_gpu_parity.py::test_stream_matches_golden runs the
pipeline on the feed).  Frames of the timed configurations and of every
content kind; a frame whose coefficient section overflows the reference's
32 Mbit feed stream falls back to the host precode with the drop rule."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check_feeds(cairo, w, h, ring, q, frames, gen, batch=0):
    ctx = cairo.Context(w, h, ring)
    ctx.set_outputs(cairo.OUT_COEF | cairo.OUT_FEED)
    if batch:
        ctx.set_batch(batch)
    tks = [ctx.submit(gen(w, h, t), t, t > 0, q) for t in range(frames)]
    for t, tk in enumerate(tks):
        out = ctx.wait(tk)
        ctx.release(tk)
        want = cairo.serialize_slice(out.table, ctx.wmb, ctx.hmb, ring, out.coef_y, out.coef_u, out.coef_v)
        assert out.feed_status == cairo.FEED_VALID, f"frame {t}: status {out.feed_status}"
        got = cairo.serialize_feed(out.feed, out.feed_bits)
        assert got[1] == want[1], f"{w}x{h} q={q} frame {t}: {got[1]} vs {want[1]} payload bits"
        assert got[0] == want[0], f"{w}x{h} q={q} frame {t}: payload differs"
    ctx.close()


@pytest.mark.parametrize("w,h,ring,q,frames", [(352, 288, 4, 16, 8), (352, 288, 2, 1, 6), (352, 288, 3, 31, 6),
                                               (200, 120, 4, 8, 5), (16, 16, 2, 16, 4), (1280, 720, 2, 16, 6),
                                               (1920, 1080, 4, 8, 4), (3840, 2160, 4, 16, 4)])
def test_feed_band4(orc, cairo, w, h, ring, q, frames):
    _check_feeds(cairo, w, h, ring, q, frames, orc.make_frame)


@pytest.mark.parametrize("kind,q", [("noise", 1), ("noise", 16), ("static", 16), ("black", 8), ("white", 31),
                                    ("ties", 1), ("pan", 16), ("gradient", 1)])
def test_feed_content(cairo, kind, q):
    from tests import content

    _check_feeds(cairo, 352, 288, 4, q, 8, lambda w, h, t: content.make(kind, w, h, t), batch=3)


def test_feed_overflow_falls_back(orc, cairo):
    """4K uniform noise at q=1: the Y coefficients of an intra frame exceed
    the 32 Mbit feed stream, whose writes the reference then drops; the frame
    is flagged and coded from its planes with the same rule, and the stream
    through the pipeline (feed outputs only) still equals the oracle's."""
    from tests import content

    w, h, ring, q = 3840, 2160, 4, 1
    ctx = cairo.Context(w, h, ring)
    ctx.set_outputs(cairo.OUT_FEED)
    rgb = content.make("noise", w, h, 0)
    tk = ctx.submit(rgb, 0, False, q)
    out = ctx.wait(tk)
    assert out.feed_status == cairo.FEED_OVERFLOW and out.coef_y is None
    cy, cu, cv = ctx.fetch_coef(tk)
    got = cairo.serialize_slice(out.table, ctx.wmb, ctx.hmb, ring, cy, cu, cv, capacity_bytes=w * h * 8)
    ctx.release(tk)
    ctx.close()
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    data, nbits = e.encode(rgb)
    head = 14 * 8 + 10 * 8  # header + frame descriptor precede the payload
    assert nbits - head == got[1]
    want = np.unpackbits(np.frombuffer(data, np.uint8), bitorder="little")[head:nbits]
    have = np.unpackbits(np.frombuffer(got[0], np.uint8), bitorder="little")[:got[1]]
    np.testing.assert_array_equal(have, want)
