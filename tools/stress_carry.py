"""Repeat test_timed_4k_many_launches' configuration (4K q=16 R=4, device
frames, feed outputs, 10 frames per launch, 44 frames) many times in one
process and compare every frame's block table and coefficient planes with the
oracle, macroblock by macroblock (tools: the r05 red-run investigation, DESIGN
§2).  The oracle streams are encoded once, on this host, before the GPU loop.

Iterations alternate the quality (--q list) so that a stale read of memory a
previous context left behind shows up as another stream's values instead of
the same ones.  A mismatch is classified per macroblock: its reference block
type (copy or coded), and whether the GPU value is zero (the fresh context's
memset), the previous frame's coefficient at the same place, or the other
quality's.

usage (GPU box): python tools/stress_carry.py [--iters 12] [--frames 44] [--batch 10] [--q 16,8]
"""
import argparse
import ctypes
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

W, H, RING = 3840, 2160, 4
WMB, HMB = W // 16, (H + 15) // 16


def oracle_stream(q, frames):
    from oracle import oracle as orc

    e = orc.OracleEncoder(RING)
    e.set_quality(q)
    out = []
    for t in range(frames):
        if t == 0:
            e.insert_intra()
        e.encode(orc.make_frame(W, H, t))
        y, u, v = (np.array(p, copy=True) for p in e.planes(1))
        out.append((np.array(e.block_table(), copy=True), y, u, v))
    return out


def mb_view_y(p):  # (HMB, WMB, 16, 16)
    return p[: HMB * 16].reshape(HMB, 16, WMB, 16).transpose(0, 2, 1, 3)


def mb_bad(got, ref):
    """Boolean (HMB, WMB): macroblocks whose Y, U or V coefficients differ."""
    by = (mb_view_y(got[0]) != mb_view_y(ref[0])).any(axis=(2, 3))
    bu = (got[1][: HMB * 8].reshape(HMB, 8, WMB, 8) != ref[1][: HMB * 8].reshape(HMB, 8, WMB, 8)).any(axis=(1, 3))
    bv = (got[2][: HMB * 8].reshape(HMB, 8, WMB, 8) != ref[2][: HMB * 8].reshape(HMB, 8, WMB, 8)).any(axis=(1, 3))
    return by | bu | bv, by, bu, bv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--frames", type=int, default=44)
    ap.add_argument("--batch", type=int, default=10)
    ap.add_argument("--q", default="16,8")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "stress_carry.json"))
    a = ap.parse_args()
    qs = [int(x) for x in a.q.split(",")]
    t0 = time.time()
    with ProcessPoolExecutor(len(qs)) as pool:
        refs = dict(zip(qs, pool.map(oracle_stream, qs, [a.frames] * len(qs))))
    print(f"[stress] oracle streams q={qs}: {time.time() - t0:.0f} s", flush=True)

    import cairo_amd
    from oracle import oracle as orc

    hip = ctypes.CDLL("libamdhip64.so.7")
    size = W * H * 3
    dev = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(a.frames * size)) == 0
    for t in range(a.frames):
        f = orc.make_frame(W, H, t)
        assert hip.hipMemcpy(ctypes.c_void_p(dev.value + t * size), f.ctypes.data_as(ctypes.c_void_p),
                             ctypes.c_size_t(size), 1) == 0
    report = {"config": {"w": W, "h": H, "ring": RING, "frames": a.frames, "batch": a.batch, "q": qs},
              "iterations": []}
    bad_total = 0
    for it in range(a.iters):
        q = qs[it % len(qs)]
        other = qs[(it + 1) % len(qs)]
        ref = refs[q]
        ctx = cairo_amd.Context(W, H, RING)
        ctx.set_outputs(cairo_amd.OUT_FEED)
        ctx.set_batch(a.batch)
        tks = [ctx.submit(dev.value + t * size, t, t != 0, q, on_device=True) for t in range(a.frames)]
        rec = {"iter": it, "q": q, "frames_bad": []}
        for t, tk in enumerate(tks):
            out = ctx.wait(tk)
            table_ok = all(np.array_equal(out.table[f], ref[t][0][f]) for f in ref[t][0].dtype.names if f != "pad")
            got = tuple(np.array(p, copy=True) for p in ctx.fetch_coef(tk))
            bad, by, bu, bv = mb_bad(got, ref[t][1:])
            if bad.any() or not table_ok:
                types = ref[t][0]["block_type"].reshape(HMB, WMB)
                copy = (types & 4) != 0
                ys, xs = np.nonzero(bad)
                gy = got[0][: HMB * 16]
                zero_y = int(sum(not mb_view_y(gy)[r, c].any() for r, c in zip(ys, xs)))
                prev_y = int(sum(t > 0 and np.array_equal(mb_view_y(gy)[r, c], mb_view_y(ref[t - 1][1])[r, c])
                                 for r, c in zip(ys, xs)))
                oth_y = int(sum(np.array_equal(mb_view_y(gy)[r, c], mb_view_y(refs[other][t][1])[r, c])
                                for r, c in zip(ys, xs)))
                d = {"frame": t, "table_ok": table_ok, "mbs_bad": int(bad.sum()), "mbs_bad_y": int(by.sum()),
                     "mbs_bad_u": int(bu.sum()), "mbs_bad_v": int(bv.sum()),
                     "bad_copy_mbs": int((bad & copy).sum()), "bad_coded_mbs": int((bad & ~copy).sum()),
                     "copy_mbs": int(copy.sum()), "bad_y_all_zero": zero_y, "bad_y_equal_prev_frame": prev_y,
                     "bad_y_equal_other_q": oth_y, "rows_bad": sorted(set(int(r) for r in ys))[:40],
                     "first": [[int(r), int(c)] for r, c in list(zip(ys, xs))[:20]]}
                rec["frames_bad"].append(d)
                print(f"[stress] iter {it} q={q} frame {t}: {json.dumps(d)}", flush=True)
            ctx.release(tk)
        ctx.sync()
        ctx.close()
        bad_total += len(rec["frames_bad"])
        report["iterations"].append(rec)
        print(f"[stress] iter {it} q={q}: {len(rec['frames_bad'])} bad frames ({time.time() - t0:.0f} s)", flush=True)
        with open(a.out, "w") as f:
            json.dump(report, f, indent=1)
    hip.hipFree(dev)
    report["bad_frames_total"] = bad_total
    with open(a.out, "w") as f:
        json.dump(report, f, indent=1)
    print(f"[stress] done: {bad_total} bad frames over {a.iters} iterations")


if __name__ == "__main__":
    main()
