"""Per-frame golden hashes of the streams bench.py times (test infrastructure).

Runs the oracle (oracle/liboracle.so, the C restatement of the reference
encoder) over one long band4 stream at a bench configuration and writes, for
every frame t, the bit count and the FNV-1a-64 of the frame's canonical
record (header/descriptor + payload, tail bits masked, header byte 7 zeroed:
oracle.canonical_frame_bytes).  bench.py and tests/test_gpu_timed.py compare
every frame the GPU encodes against these without running the oracle on the
GPU box (about 3.5 s per 4K frame on one core).

The stream is exactly what bench.py submits: frame t is make_band4(w, h, t)
(seed 1234) -- or bench.content_frame(content, w, h, t) for --content noise /
static -- frame 0 intra, every later frame a P-frame, quality and ring of the
config (bench.CONFIGS).  The file is rewritten every `--flush` frames, so
a partial run leaves a usable prefix.

usage: python tests/golden/make_stream_golden.py --config 4k --frames 1440 [--content noise]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as orc  # noqa: E402

# name: (width, height, ring, quality) -- bench.CONFIGS
CONFIGS = {
    "4k": (3840, 2160, 4, 16),
    "1080p": (1920, 1080, 4, 8),
    "720p": (1280, 720, 2, 16),
    "cif": (352, 288, 4, 16),
}


def path_for(config: str, q: int | None = None, content: str = "band4") -> str:
    w, h, ring, q0 = CONFIGS[config]
    sfx = "" if content == "band4" else f"_{content}"
    return os.path.join(HERE, f"stream_{config}_q{q if q is not None else q0}_r{ring}{sfx}.json")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="4k", choices=sorted(CONFIGS))
    p.add_argument("--frames", type=int, default=1440)
    p.add_argument("--quality", type=int, default=None)
    p.add_argument("--flush", type=int, default=16)
    p.add_argument("--content", default="band4", choices=["band4", "noise", "static"])
    a = p.parse_args()
    w, h, ring, q = CONFIGS[a.config]
    if a.quality is not None:
        q = a.quality
    out = path_for(a.config, q, a.content)
    from bench import content_frame
    e = orc.OracleEncoder(ring)
    e.set_quality(q)
    bits, fnv = [], []
    t0 = time.time()

    def dump(final):
        doc = {"_source": "oracle/evx_oracle.c via tests/golden/make_stream_golden.py",
               "config": a.config, "width": w, "height": h, "ring": ring, "quality": q,
               "content": a.content, "seed": 1234 if a.content != "noise" else 7, "first_intra": True,
               "hash": "fnv1a64 of oracle.canonical_frame_bytes(record, bits, t == 0), per frame",
               "frames": len(bits), "complete": final, "frame_bits": bits, "frame_fnv1a64": fnv}
        tmp = out + ".tmp"
        with open(tmp, "w") as f:
            json.dump(doc, f, separators=(",", ":"))
        os.replace(tmp, out)

    for t in range(a.frames):
        data, n = e.encode(content_frame(a.content, w, h, t))
        bits.append(int(n))
        fnv.append(f"{orc.fnv1a64(orc.canonical_frame_bytes(data, n, t == 0)):016x}")
        if (t + 1) % a.flush == 0:
            dump(False)
            print(f"{a.config}: {t + 1} frames, {time.time() - t0:.0f} s", flush=True)
    dump(True)
    print("wrote", out, flush=True)


if __name__ == "__main__":
    main()
