"""Rate-distortion + throughput sweep over the quality (BASELINE.json configs[4]:
3840x2160 p-frames, quality 1..31, VAQ on, one MI355X).

Per quality q, on the band4 content (seed 1234), ring R = 4:
  * hot-path throughput: `--frames` P-frames after 16 warm-up frames, inputs
    resident in HBM, timed like bench.py (Mpix/s);
  * rate: payload bits per P-frame through the native frame pipeline (host
    entropy), plus the 10-byte frame descriptor the encoder writes per frame;
  * distortion: PSNR (peak 255) of the last frame's deblocked reconstruction
    against its converted source, luma and chroma separately.
  * parity: the canonical FNV-1a-64 (tail bits and header byte 7 masked) of
    every frame's stream record that the oracle's golden stream of this quality
    covers (tests/golden/stream_4k_q<q>_r4.json, made off-box by
    tests/golden/make_stream_golden.py: 40 frames, all three references live
    from frame 3) is compared here, and the hashes are kept in the row, so that
    tests/test_rd_sweep_pinned.py ties the committed table to the goldens and
    the goldens to the oracle (this tool uses the oracle library only for its
    FNV-1a-64, never its encoder).
Writes one JSON object per q to stdout and the whole table to --out.
usage (GPU box): python tools/rd_sweep.py [--config 4k] [--frames 48] [--q 1,4,8,...]
"""
import argparse
import hashlib
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (CONFIGS, run_hot_path)


def psnr(a, b):
    mse = float(np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2))
    return float("inf") if mse == 0 else 10.0 * math.log10(255.0 ** 2 / mse)


def record_hashes(w, h, ring, q, t, payload, nbits):
    """Canonical SHA-256 (16 hex digits) and FNV-1a-64 of frame t's stream
    record: header or descriptor + payload, bits beyond the end and header
    byte 7 zeroed (oracle.canonical_frame_bytes), and its bit count."""
    import cairo_amd
    from oracle import oracle as orc

    rec, n = bench.record(cairo_amd, w, h, ring, q, t, payload, nbits)
    b = orc.canonical_frame_bytes(rec, n, t == 0)
    return hashlib.sha256(b).hexdigest()[:16], f"{orc.fnv1a64(b):016x}", n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4k", choices=sorted(bench.CONFIGS))
    ap.add_argument("--frames", type=int, default=160, help="timed P-frames per quality")
    ap.add_argument("--q", default=",".join(str(q) for q in range(1, 32)))
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "rd_sweep.json"))
    ap.add_argument("--check", type=int, default=8,
                    help="frames per quality also pinned by SHA-256 (SURVEY §8(d) Config 5: >= 8)")
    a = ap.parse_args()
    import torch

    import cairo_amd

    w, h, ring, _, _ = bench.CONFIGS[a.config]
    ring = 4
    warm = 16
    n = warm + a.frames
    host = np.empty((n, h, w, 3), np.uint8)
    for f in range(n):
        host[f] = cairo_amd.make_band4(w, h, f)
    frames = torch.from_numpy(host).to("cuda:0")
    base, stride = frames.data_ptr(), w * h * 3

    def ptr(f):
        return base + f * stride

    rows = []
    for q in [int(x) for x in a.q.split(",")]:
        # throughput (hot path)
        ctx = cairo_amd.Context(w, h, ring)
        ctx.set_outputs(cairo_amd.OUT_FEED)  # as bench.py's timed context
        stages = ctx.stages
        bench.run_hot_path(ctx, ptr, 0, warm, q, stages)
        ctx.sync()
        t0 = time.perf_counter()
        bench.run_hot_path(ctx, ptr, warm, a.frames, q, stages)
        ctx.sync()
        el = time.perf_counter() - t0
        ctx.close()
        # rate and distortion (frame pipeline: entropy on host threads)
        ctx = cairo_amd.Context(w, h, ring)
        st = cairo_amd.Stream(ctx, threads=14)
        tks = []
        bits = []
        pins = []
        gold = bench.golden_stream(a.config, "band4", q, ring)
        ncheck = min(n, gold["frames"]) if gold else 0
        fnv = []

        def take(tk):
            data, nb = st.collect(tk)
            t = len(bits)
            bits.append(nb)
            if t < max(a.check, ncheck):
                sha, h64, rec_bits = record_hashes(w, h, ring, q, t, data, nb)
                if t < a.check:
                    pins.append({"frame": t, "record_bits": rec_bits, "sha256_16": sha})
                if t < ncheck:
                    fnv.append(h64)

        for f in range(n):
            tks.append(st.submit(ptr(f), f, f > 0, q, on_device=True))
            if len(tks) == stages:
                take(tks.pop(0))
        while tks:
            take(tks.pop(0))
        st.close()
        last = n - 1
        src = ctx.read_planes(0)
        rec = ctx.read_planes(2 + last % ring)
        ctx.close()
        hh, ww = h, w  # nominal area (the padding rows/columns are not part of the picture)
        pb = bits[1:]
        row = {"quality": q, "mpix_per_s": round(w * h * a.frames / el / 1e6, 1),
               "p_frame_kbytes": round((float(np.mean(pb)) / 8 + 10) / 1e3, 2),
               "bits_per_pixel": round(float(np.mean(pb)) / (w * h), 4),
               "i_frame_kbytes": round((bits[0] / 8 + 24) / 1e3, 2),
               "psnr_y": round(psnr(src[0][:hh, :ww], rec[0][:hh, :ww]), 2),
               "psnr_u": round(psnr(src[1][:hh // 2, :ww // 2], rec[1][:hh // 2, :ww // 2]), 2),
               "psnr_v": round(psnr(src[2][:hh // 2, :ww // 2], rec[2][:hh // 2, :ww // 2]), 2),
               "pinned_frames": pins}
        mism = [t for t in range(ncheck) if fnv[t] != gold["frame_fnv1a64"][t]]
        row["golden"] = {"path": gold["path"] if gold else None, "frames_checked": ncheck,
                         "mismatches": len(mism), "mismatched_frames": mism, "frame_fnv1a64": fnv}
        rows.append(row)
        print(json.dumps(row), flush=True)
    out = {"config": f"{w}x{h} p-frames, ring R={ring}, band4 seed 1234 (BASELINE.json configs[4])",
           "timed_p_frames_per_quality": a.frames, "rows": rows}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
