"""The committed quality sweep (BASELINE.json configs[4]) against
the oracle: tools/rd_sweep.py records, per quality, the canonical SHA-256 of
the stream records of the first frames its GPU frame pipeline produced; here
the oracle (oracle/evx_oracle.c, the checker) encodes the same band4 frames at
the same quality on the CPU and must give the same records, bit for bit.
So the table's rates come from streams that are the reference's."""
import glob
import hashlib
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _sweep():
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_4k_rd_sweep.json")), reverse=True):
        d = json.load(open(path))
        if d.get("rows") and all(r.get("pinned_frames") for r in d["rows"]):
            return path, d
    return None, None


PATH, SWEEP = _sweep()
ROWS = SWEEP["rows"] if SWEEP else []
MIN_PINNED = 8  # SURVEY.md §8(d) Config 5: >= 8 frames per quality (all three references live from frame 3)


def _oracle_records(q, n):
    """(record bits, canonical SHA-256/16) of band4 frames 0..n-1 at quality q
    through the oracle (one process per quality)."""
    import sys

    sys.path.insert(0, ROOT)
    import cairo_amd
    from oracle import oracle as orc

    w, h, ring = 3840, 2160, 4
    enc = orc.OracleEncoder(ring)
    enc.set_quality(q)
    out = []
    for t in range(n):
        data, nbits = enc.encode(cairo_amd.make_band4(w, h, t))
        out.append((nbits, hashlib.sha256(orc.canonical_frame_bytes(data, nbits, t == 0)).hexdigest()[:16]))
    return out


@pytest.mark.skipif(SWEEP is None, reason="no committed 4K quality sweep with pinned frames")
def test_sweep_records_match_oracle():
    """Every quality of the committed sweep: at least MIN_PINNED frames pinned
    (frames 0..n-1, so the steady state with three live references is
    covered), each equal to the oracle's record.  The qualities run in
    parallel processes (about 3.5 s of oracle per 4K frame here)."""
    from concurrent.futures import ProcessPoolExecutor

    assert [r["quality"] for r in ROWS] == [1, 2, 4, 8, 12, 16, 20, 24, 28, 31]
    jobs = {}
    for row in ROWS:
        pins = sorted(row["pinned_frames"], key=lambda p: p["frame"])
        assert [p["frame"] for p in pins] == list(range(len(pins)))
        assert len(pins) >= MIN_PINNED, f"{os.path.basename(PATH)} q={row['quality']}: {len(pins)} frames pinned"
        jobs[row["quality"]] = pins
    with ProcessPoolExecutor(min(len(jobs), max(1, os.cpu_count() or 1))) as pool:
        futs = {q: pool.submit(_oracle_records, q, len(p)) for q, p in jobs.items()}
        for q, pins in jobs.items():
            got = futs[q].result()
            for p, (nbits, sha) in zip(pins, got):
                assert (nbits, sha) == (p["record_bits"], p["sha256_16"]), \
                    f"{os.path.basename(PATH)} q={q} frame {p['frame']}"
