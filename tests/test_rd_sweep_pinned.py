"""The committed quality sweep (BASELINE.json configs[4]) against
the oracle.

tools/rd_sweep.py, on the GPU box, compares the canonical FNV-1a-64 of every
stream record its frame pipeline produced with the oracle's golden stream of
the same quality (tests/golden/stream_4k_q<q>_r4.json, 40 frames each, made in
the build container by tests/golden/make_stream_golden.py) and keeps the
hashes in its row.  Here, on the CPU:
  * the committed table covers q = 1..31, each quality with >= MIN_FRAMES
    frames (all three references live from frame 3) checked on the box with no
    mismatch, and its recorded hashes equal the committed goldens;
  * the goldens are the oracle's: the first frames of every quality are
    re-encoded by the oracle (oracle/evx_oracle.c, the checker) and must hash
    the same.
So the table's rates and PSNRs come from streams that are the reference's."""
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
QUALITIES = list(range(1, 32))
MIN_FRAMES = 35  # frames per quality compared with the oracle on the box
REENCODE = 2  # frames per quality re-encoded here by the oracle (about 3.7 s each)


def _sweep():
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_4k_rd_sweep.json")), reverse=True):
        d = json.load(open(path))
        if d.get("rows") and all("golden" in r for r in d["rows"]):
            return path, d
    return None, None


PATH, SWEEP = _sweep()


def _golden(q):
    return json.load(open(os.path.join(GOLDEN, f"stream_4k_q{q}_r4.json")))


def _oracle_fnv(q, n):
    """FNV-1a-64 of the canonical records of band4 frames 0..n-1 at quality q
    through the oracle (one process per quality)."""
    import sys

    sys.path.insert(0, ROOT)
    import cairo_amd
    from oracle import oracle as orc

    enc = orc.OracleEncoder(4)
    enc.set_quality(q)
    out = []
    for t in range(n):
        data, nbits = enc.encode(cairo_amd.make_band4(3840, 2160, t))
        out.append((int(nbits), f"{orc.fnv1a64(orc.canonical_frame_bytes(data, nbits, t == 0)):016x}"))
    return out


def test_golden_streams_cover_every_quality():
    for q in QUALITIES:
        g = _golden(q)
        assert (g["width"], g["height"], g["ring"], g["quality"], g["content"]) == (3840, 2160, 4, q, "band4")
        assert g["frames"] >= MIN_FRAMES and len(g["frame_fnv1a64"]) == g["frames"], f"q={q}"


@pytest.mark.skipif(SWEEP is None, reason="no committed 4K quality sweep with golden checks")
def test_sweep_rows_checked_against_goldens():
    rows = SWEEP["rows"]
    assert [r["quality"] for r in rows] == QUALITIES
    for r in rows:
        q, g = r["quality"], r["golden"]
        name = f"{os.path.basename(PATH)} q={q}"
        assert g["frames_checked"] >= MIN_FRAMES, name
        assert g["mismatches"] == 0 and not g["mismatched_frames"], name
        assert g["frame_fnv1a64"] == _golden(q)["frame_fnv1a64"][: g["frames_checked"]], name


def test_goldens_are_the_oracles():
    """Every quality's golden stream starts with the oracle's own records (the
    qualities in parallel processes)."""
    from concurrent.futures import ProcessPoolExecutor

    with ProcessPoolExecutor(max(1, min(len(QUALITIES), os.cpu_count() or 1))) as pool:
        futs = {q: pool.submit(_oracle_fnv, q, REENCODE) for q in QUALITIES}
        for q, fut in futs.items():
            g = _golden(q)
            for t, (nbits, h) in enumerate(fut.result()):
                assert (nbits, h) == (g["frame_bits"][t], g["frame_fnv1a64"][t]), f"q={q} frame {t}"
