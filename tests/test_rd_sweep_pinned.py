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


@pytest.mark.skipif(SWEEP is None, reason="no committed 4K quality sweep with pinned frames")
@pytest.mark.parametrize("row", ROWS, ids=lambda r: f"q{r['quality']}")
def test_sweep_records_match_oracle(row):
    import cairo_amd
    from oracle import oracle as orc

    w, h, ring, q = 3840, 2160, 4, row["quality"]
    enc = orc.OracleEncoder(ring)
    enc.set_quality(q)
    pins = sorted(row["pinned_frames"], key=lambda p: p["frame"])
    assert [p["frame"] for p in pins] == list(range(len(pins)))
    for p in pins:
        t = p["frame"]
        data, nbits = enc.encode(cairo_amd.make_band4(w, h, t))
        sha = hashlib.sha256(orc.canonical_frame_bytes(data, nbits, t == 0)).hexdigest()[:16]
        assert (nbits, sha) == (p["record_bits"], p["sha256_16"]), f"{os.path.basename(PATH)} q={q} frame {t}"
