"""Time the host entropy stage (cairo_serialize_slice) on one core.

The block table and coefficients come from the CPU oracle encoding band4
frames (I, P, P, ...), so the statistics are the bench's; the oracle is only
the input generator here.  Prints ms per frame.

    python tools/entropy_bench.py [--w 1280 --h 720 --ring 2 --q 16 --reps 20]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import cairo_amd  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--w", type=int, default=1280)
    p.add_argument("--h", type=int, default=720)
    p.add_argument("--ring", type=int, default=2)
    p.add_argument("--q", type=int, default=16)
    p.add_argument("--frames", type=int, default=3)
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    e = orc.OracleEncoder(a.ring)
    e.set_quality(a.q)
    wmb, hmb = (a.w + 15) // 16, (a.h + 15) // 16
    for t in range(a.frames):
        data, nbits = e.encode(orc.make_frame(a.w, a.h, t))
    y, u, v = (x.copy() for x in e.planes(1))
    table = e.block_table().copy()
    pay, pbits = cairo_amd.serialize_slice(table, wmb, hmb, a.ring, y, u, v)
    assert pbits == nbits - 80, (pbits, nbits)
    best = 1e9
    for _ in range(a.reps):
        t0 = time.perf_counter()
        cairo_amd.serialize_slice(table, wmb, hmb, a.ring, y, u, v)
        best = min(best, time.perf_counter() - t0)
    print(f"{a.w}x{a.h} q={a.q} R={a.ring}: payload {pbits} bits, {best * 1e3:.3f} ms per frame (best of {a.reps})")


if __name__ == "__main__":
    main()
