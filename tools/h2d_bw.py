"""Pinned host -> device copy bandwidth on this box, without the engine: the
ceiling of bench.py's host_rgb leg (one 4K RGB frame = 24.9 MB per copy).
usage: python tools/h2d_bw.py [--mb 24.9] [--copies 200]"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=24.8832)
    ap.add_argument("--copies", type=int, default=200)
    a = ap.parse_args()
    n = int(a.mb * 1e6)
    host = [torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(4)]
    dev = [torch.empty(n, dtype=torch.uint8, device="cuda:0") for _ in range(4)]
    s = torch.cuda.Stream()
    out = {}
    for label, stream in (("default_stream", torch.cuda.current_stream()), ("side_stream", s)):
        with torch.cuda.stream(stream):
            for i in range(8):
                dev[i % 4].copy_(host[i % 4], non_blocking=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.copies):
                dev[i % 4].copy_(host[i % 4], non_blocking=True)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        out[label] = {"GBps": round(n * a.copies / el / 1e9, 2), "ms_per_copy": round(el / a.copies * 1e3, 3)}
    d2h = torch.empty(n, dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.copies // 2):
        d2h.copy_(dev[i % 4], non_blocking=True)
    torch.cuda.synchronize()
    out["d2h"] = {"GBps": round(n * (a.copies // 2) / (time.perf_counter() - t0) / 1e9, 2)}
    out["bytes_per_copy"] = n
    print(json.dumps(out))


if __name__ == "__main__":
    main()
