"""Frame-interleaved group parity worker (run by tests/test_gpu_group.py in a
subprocess, GPU test infrastructure).

  inproc: N member contexts in this process on one device (the multi-GPU
          protocol emulated on one GPU); this process needs
          GPU_MAX_HW_QUEUES >= 3 N (each member's two launch streams and copy
          stream on hardware queues of their own: a launch queued behind
          another member's on a shared queue would wait for it).
  xproc:  this process is member RANK of N processes on one device, sharing
          its buffers through IPC handles (cross_device records: fine-grained
          memory, system-scope hand-offs), records exchanged over gloo.

Every frame's block table and coefficients and the final reconstructions are
compared with the oracle encoding the same stream in one context.  Prints
one JSON line; exit status 0 = bit-exact.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import cairo_amd  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def payload_bits(out, ctx, ring, tk):
    """The frame's payload from its feed (or planes), as a bit array."""
    if out.feed_status == cairo_amd.FEED_VALID:
        data, n = cairo_amd.serialize_feed(out.feed, out.feed_bits)
    else:
        cy, cu, cv = (out.coef_y, out.coef_u, out.coef_v) if out.coef_y is not None else ctx.fetch_coef(tk)
        data, n = cairo_amd.serialize_slice(out.table, ctx.wmb, ctx.hmb, ring, cy, cu, cv)
    return np.unpackbits(np.frombuffer(data, np.uint8), bitorder="little")[:n]


def table_mismatch(a, b):
    return [f for f in a.dtype.names if f != "pad" and not np.array_equal(a[f], b[f])]


def oracle_stream(w, h, ring, q, frames, intra_every):
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    ref = []
    for t in range(frames):
        intra = t == 0 or (intra_every and t % intra_every == 0)
        if intra:
            e.insert_intra()
        data, n = e.encode(orc.make_frame(w, h, t))
        head = (14 * 8 if t == 0 else 0) + 10 * 8  # header + frame descriptor precede the payload
        bits = np.unpackbits(np.frombuffer(data, np.uint8), bitorder="little")[head:n]
        ref.append((intra, e.block_table(), e.planes(1), bits))
    final = {t: e.planes(2 + t % ring) for t in range(max(0, frames - ring), frames)}
    return ref, final


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["inproc", "xproc"])
    ap.add_argument("--members", type=int, default=2)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--store", default="")
    ap.add_argument("--w", type=int, default=352)
    ap.add_argument("--h", type=int, default=288)
    ap.add_argument("--ring", type=int, default=4)
    ap.add_argument("--q", type=int, default=16)
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--intra-every", type=int, default=0)
    ap.add_argument("--rejoin", type=int, default=0, help="inproc: reset, rejoin and encode the stream again, N times")
    ap.add_argument("--feed", action="store_true", help="members hand over GPU-precoded feeds (bench's mode); "
                                                         "payloads are checked too")
    a = ap.parse_args()
    w, h, ring, q, F, N = a.w, a.h, a.ring, a.q, a.frames, a.members
    ref, final = oracle_stream(w, h, ring, q, F, a.intra_every)
    bad = []
    if a.mode == "inproc":
        g = cairo_amd.Group(w, h, ring, [0] * N, batch=a.batch)
        assert F <= N * g.stages  # every frame in flight at once
        for rnd in range(1 + a.rejoin):
            if rnd:  # reset every member and rejoin: a new stream from frame 0
                g.reset()
            for t in range(F):
                g.submit(orc.make_frame(w, h, t), t, not ref[t][0], q)
            for t in range(F):
                out = g.wait(t)
                if table_mismatch(out.table, ref[t][1]) or any(
                        not np.array_equal(x, y) for x, y in zip((out.coef_y, out.coef_u, out.coef_v), ref[t][2])):
                    bad.append(f"{t}" + (f" (after rejoin {rnd})" if rnd else ""))
                g.release(t)
            for t, planes in final.items():
                if any(not np.array_equal(x, y) for x, y in zip(g.recon(t), planes)):
                    bad.append(f"recon {t}" + (f" (after rejoin {rnd})" if rnd else ""))
        g.close()
    else:
        import torch.distributed as dist

        dist.init_process_group("gloo", init_method=f"file://{a.store}", rank=a.rank, world_size=N)
        ctx = cairo_amd.Context(w, h, ring)  # the library's default staging slots (96)
        ctx.set_batch(a.batch)
        if a.feed:
            ctx.set_outputs(cairo_amd.OUT_FEED)
        ctx.set_workgroups(max(1, ctx.max_workgroups() // N))  # N members share the device
        recs = [None] * N
        rec = ctx.peer_info(cross_device=True)
        if ctx.stages * ctx.wa * ctx.ha * 3 >= 1 << 31:  # the export is chunked below 1 GiB per allocation
            assert int.from_bytes(rec[28:32], "little") >= 2, "output_cache exported in one allocation"
        dist.all_gather_object(recs, rec)
        ctx.join_group(a.rank, recs)
        mine = [t for t in range(F) if t % N == a.rank]
        frames = {t: orc.make_frame(w, h, t) for t in mine}
        dist.barrier()  # every member ready: in-kernel waits on the others are bounded (2 s)
        tk = {t: ctx.submit(frames[t], t, not ref[t][0], q) for t in mine}
        ctx.flush()
        for t in mine:
            out = ctx.wait(tk[t])
            if table_mismatch(out.table, ref[t][1]):
                bad.append(t)
            elif a.feed:
                if not np.array_equal(payload_bits(out, ctx, ring, tk[t]), ref[t][3]):
                    bad.append(f"payload {t}")
            elif any(not np.array_equal(x, y) for x, y in zip((out.coef_y, out.coef_u, out.coef_v), ref[t][2])):
                bad.append(t)
            ctx.release(tk[t])
        ctx.sync()
        dist.barrier()  # every member's frames encoded: their pushes into this member's mirrors are done
        for t, planes in final.items():  # its own frames, and the mirrors other members pushed here
            lay = cairo_amd.group_layout(t, N, ring, ctx.stages, mirror=True)
            if lay["member"] == a.rank or a.rank in lay["readers"]:
                got = ctx.read_planes(2 + lay["recon_slot"])
                if any(not np.array_equal(x, y) for x, y in zip(got, planes)):
                    bad.append(f"recon {t}" + ("" if lay["member"] == a.rank else " (mirror)"))
        dist.barrier()  # the others may still read this member's buffers until they finish
        ctx.close()
        dist.destroy_process_group()
    print(json.dumps({"mode": a.mode, "rank": a.rank, "members": N, "frames": F, "mismatched": bad}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
