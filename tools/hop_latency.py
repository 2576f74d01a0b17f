"""Hop latency of the progress-word hand-off on one MI355X:
runs tools/bin/hop_latency (make builds it) in its local modes and as a pair of
processes, for a few payload sizes, and writes one JSON document.

This parent never touches the GPU; each measurement is a child process with a
time limit of its own.
usage (GPU box): python tools/hop_latency.py [--iters 4000] [--out gpurun_out/hop_latency.json]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "bin", "hop_latency")


def run(args, timeout=60):
    r = subprocess.run([BIN] + args, capture_output=True, text=True, timeout=timeout)
    if r.returncode:
        raise RuntimeError(f"{args}: rc {r.returncode}: {r.stderr.strip()[-400:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def pair(payload, iters, timeout=60):
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "handle")
        ping = subprocess.Popen([BIN, "ping", f, str(payload), str(iters)], stdout=subprocess.PIPE,
                                stderr=subprocess.PIPE, text=True)
        pong = subprocess.Popen([BIN, "pong", f, str(payload), str(iters)], stdout=subprocess.PIPE,
                                stderr=subprocess.PIPE, text=True)
        try:
            out, err = ping.communicate(timeout=timeout)
            pong.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            ping.kill()
            pong.kill()
            raise
        if ping.returncode or pong.returncode:
            raise RuntimeError(f"pair rc {ping.returncode}/{pong.returncode}: {err.strip()[-400:]}")
        return json.loads(out.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=4000)
    ap.add_argument("--payloads", default="0,4096,16384")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "hop_latency.json"))
    a = ap.parse_args()
    rows = []
    for pay in [int(x) for x in a.payloads.split(",")]:
        for scope in ("agent", "system"):
            for xcd in ("same", "cross"):
                rows.append(run(["local", scope, xcd, str(pay), str(a.iters)]))
                print(json.dumps(rows[-1]), flush=True)
        rows.append(pair(pay, a.iters))
        print(json.dumps(rows[-1]), flush=True)
    stale = [run(["stale", kind, "4096"]) for kind in ("sc1", "plain")]
    for r in stale:
        print(json.dumps(r), flush=True)
    doc = {"what": "one progress-word hop (producer: payload stores, vmcnt(0), barrier, release fence, word; "
                   "consumer: poll, acquire fence, payload loads), ping-pong between two 256-thread workgroups, "
                   "round trip / 2, s_memrealtime; one MI355X (no xGMI link in the path)",
           "iters": a.iters, "rows": rows,
           "stale_line_probe": stale}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(doc, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
