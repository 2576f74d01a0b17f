"""Regenerate tests/golden/oracle_streams.json from the oracle (oracle/liboracle.so).

The oracle itself is pinned against the reference outputs recorded in
SURVEY.md §8(c) (tests/golden/survey_cif.json, tests/test_oracle.py).  This
file freezes the oracle's full canonical stream hashes (FNV-1a-64 over each
frame's bytes, tail bits masked, header byte 7 zeroed, chained over frames)
so GPU parity tests can check whole streams without re-running the oracle.

usage: python tests/golden/make_golden.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as orc  # noqa: E402

CONFIGS = [
    # name, w, h, ring, quality, intra_only, frames
    ("cif_q16_ionly_r4", 352, 288, 4, 16, True, 10),
    ("cif_q16_ippp_r4", 352, 288, 4, 16, False, 10),
    ("cif_q16_ippp_r2", 352, 288, 2, 16, False, 10),
    ("cif_q8_ippp_r4", 352, 288, 4, 8, False, 10),
    ("cif_q1_ippp_r4", 352, 288, 4, 1, False, 10),
    ("cif_q31_ippp_r4", 352, 288, 4, 31, False, 10),
    ("odd_200x120_q16_r3", 200, 120, 3, 16, False, 6),
    ("hd720_q16_ippp_r2", 1280, 720, 2, 16, False, 4),
    ("hd1080_q8_ippp_r4", 1920, 1080, 4, 8, False, 3),
]


def run(name, w, h, ring, q, intra_only, frames):
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    bits, hsh, total = [], orc.FNV_OFFSET, 0
    for t in range(frames):
        if intra_only:
            e.insert_intra()
        data, n = e.encode(orc.make_frame(w, h, t))
        b = orc.canonical_frame_bytes(data, n, t == 0)
        hsh = orc.fnv1a64(b, hsh)
        bits.append(n)
        total += len(b)
    return {"name": name, "width": w, "height": h, "ring": ring, "quality": q,
            "intra_only": intra_only, "frames": frames, "frame_bits": bits,
            "total_bytes": total, "fnv1a64": f"{hsh:016x}"}


if __name__ == "__main__":
    out = {"_source": "oracle/evx_oracle.c via tests/golden/make_golden.py", "seed": 1234,
           "content": "band4", "configs": [run(*c) for c in CONFIGS]}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_streams.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)
