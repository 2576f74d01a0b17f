"""One 4K stream over N GPUs: a model of the two partitions, from
quantities measured on one MI355X.

Inputs (defaults: the round-6 measurements, DESIGN §6 "Hop latency and the
partition model"):
  --t1       engine ms per 4K frame on one GPU, throughput-bound (bench.py)
  --lag-idle the dependency lag between consecutive frames (us): frame j+1's
             macroblock (x, 0) coded behind frame j's (tools/k2_phases.py,
             4K, top row, 4 frames in flight: the GPU far from full)
  --lag-full the same with 32 frames in flight (a full GPU)
  --hop      one progress-word hop with the deblock chunk's mirror push (us,
             tools/hop_latency.py: cross-process, system scope, 4 KB payload)
  --hop0     one hop without payload (a granule or flag hand-off)
  --xgmi     extra latency per cross-GPU hop for the xGMI link (not
             measurable on a one-GPU box: a list of values to bracket it)

Model.  The lag grows with a GPU's load u (0 idle .. 1 full) as
lag(u) = lag_idle + (lag_full - lag_idle) u.  A stream's frame rate F is bounded by
  * throughput: F <= N / (T1 * imbalance)  (imbalance 1 for whole frames,
    ceil(135 / N) * N / 135 for row shards of the 135 macroblock rows);
  * the lag chain: consecutive frames start at least L = lag(u) + hops
    apart, hops being what the chain crosses between GPUs per frame:
      - frame interleave (built): frame n+1 waits on frame n's progress
        word, on another GPU: one hop with the mirror push;
      - row shard (north_star): within a shard the chain is local, but the
        chain of every frame crosses each boundary twice (the intra search's
        granules of the row above, A9, and the deblock's rewrite of the
        rows above the boundary, A20, which the next frame waits for): two
        hops (one granule, one with payload);
      - hybrid (inter search sharded, the coding wavefront and deblock on one
        GPU): the one GPU's coder pool is the bound, F <= 1 / coder time per
        frame with every slot a coder.
  with u = F * T1 * imbalance / N (the load each GPU carries).  F solves the
  fixed point min(throughput, 1 / L(u(F))).
usage: python tools/scaling_model.py [--json out.json]
"""
import argparse
import json
import math


def solve(n, t1_ms, lag_idle, lag_full, hops_us, imbalance=1.0):
    """Frames/s of the fixed point F = min(N / (T1 imb), 1 / L(u(F)))."""
    cap = n / (t1_ms * 1e-3 * imbalance)
    lo, hi = 0.0, cap
    for _ in range(200):  # bisection on F - min(cap, 1/L(F)) (monotone)
        f = 0.5 * (lo + hi)
        u = min(1.0, f * t1_ms * 1e-3 * imbalance / n)
        lag_s = (lag_idle + (lag_full - lag_idle) * u + hops_us) * 1e-6
        if f <= min(cap, 1.0 / lag_s):
            lo = f
        else:
            hi = f
    return lo, cap


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--t1", type=float, default=1.233)
    ap.add_argument("--lag-idle", type=float, default=180.0)
    ap.add_argument("--lag-full", type=float, default=290.0)
    ap.add_argument("--hop", type=float, default=1.98)
    ap.add_argument("--hop0", type=float, default=0.74)
    ap.add_argument("--coder-full-ms", type=float, default=0.0,
                    help="hybrid bound: ms per frame of the coding wavefront with every slot a coder "
                         "(default: T1 * coder share of the slots)")
    ap.add_argument("--xgmi", default="0,2,5")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    rows = []
    one = solve(1, a.t1, a.lag_idle, a.lag_full, 0.0)[0]
    coder_full = a.coder_full_ms or a.t1 * 184.0 / 384.0  # 184 of 384 slots per launch are coders at 4K
    for x in [float(v) for v in a.xgmi.split(",")]:
        for n in (1, 2, 4, 8):
            hi = 0.0 if n == 1 else a.hop + x
            fi, capi = solve(n, a.t1, a.lag_idle, a.lag_full, hi)
            imb = math.ceil(135 / n) * n / 135
            hr = 0.0 if n == 1 else (a.hop0 + x) + (a.hop + x)
            fr, capr = solve(n, a.t1, a.lag_idle, a.lag_full, hr, imb)
            fh = one if n == 1 else min(1e3 / coder_full, solve(n, a.t1, a.lag_idle, a.lag_full, a.hop + x)[0])
            rows.append({"xgmi_us": x, "gpus": n,
                         "interleave_fps": round(fi), "interleave_x": round(fi / one, 2),
                         "interleave_bound": "throughput" if fi >= 0.999 * capi else "lag",
                         "row_shard_fps": round(fr), "row_shard_x": round(fr / one, 2),
                         "row_shard_bound": "throughput" if fr >= 0.999 * capr else "lag",
                         "hybrid_fps": round(fh), "hybrid_x": round(fh / one, 2)})
    out = {"inputs": vars(a), "one_gpu_fps": round(one), "rows": rows}
    print(json.dumps(out, indent=1))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
