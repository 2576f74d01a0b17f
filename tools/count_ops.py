"""Algorithmic pixel-op counts per frame -> profiles/algorithmic_ops.json.

The oracle (test infrastructure: the C restatement of the reference encoder)
counts the macroblock-sized SAD, MAD, zero-SAD and lerp evaluations the
reference's searches make (motion.cpp:111-494); a pixel-op is one
abs-difference, max or lerp per pixel (256 per SAD, 384 per MAD and per lerp).
This is the work the reference algorithm defines, independent of how the GPU
schedules it; bench.py divides it by the engine's busy time for its VALU
roofline line.  band4 content, seed 1234, the BASELINE configs.
usage: python tools/count_ops.py [--frames 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import CONFIGS  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--configs", default="720p,1080p,4k")
    ap.add_argument("--content", default="band4", choices=["band4", "noise", "static"],
                    help="bench.py --content (keys other than band4 get a _<content> suffix)")
    a = ap.parse_args()
    from bench import content_frame
    out_path = os.path.join(ROOT, "profiles", "algorithmic_ops.json")
    res = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for name in a.configs.split(","):
        w, h, ring, q, idx = CONFIGS[name]
        e = orc.OracleEncoder(ring)
        e.set_quality(q)
        per = []
        for t in range(a.frames):
            orc.op_counts(reset=True)
            e.encode(content_frame(a.content, w, h, t))
            per.append(orc.op_counts())
        p = [c["pixel_ops"] for c in per[1:]]
        mbs = ((w + 15) // 16) * ((h + 15) // 16)
        key = name if a.content == "band4" else f"{name}_{a.content}"
        res[key] = {"content": a.content, "width": w, "height": h, "ring": ring, "quality": q, "baseline_config": idx,
                     "frames": a.frames, "per_frame": per,
                     "pixel_ops_per_p_frame": int(sum(p) / len(p)),
                     "pixel_ops_per_mb": round(sum(p) / len(p) / mbs, 1)}
        print(key, res[key]["pixel_ops_per_p_frame"], res[key]["pixel_ops_per_mb"], flush=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
