"""Blit-kernel copies inside bench.py's timed region, from a rocprofv3 kernel
trace (run on the GPU box: rocprofv3 --kernel-trace --memory-copy-trace
--output-format csv -d <dir> -o run -- python3 bench.py ...).

The timed region spans the engine launches after the warm-up ones: launch
index >= warmup (bench.py --warmup, 3 by default), through the end of the last
engine launch.  Prints the number and the total duration of
__amd_rocclr_copyBuffer (shader blit) dispatches, of __amd_rocclr_fillBuffer
(memset) dispatches, and of SDMA memory copies
(memory-copy trace) that start inside it, and the same over the whole run.
usage: python tools/trace_copies.py <dir with run_kernel_trace.csv> [--warmup 3]
"""
import argparse
import csv
import glob
import json
import os


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    kt = rows(a.dir, "*kernel_trace.csv")
    eng = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kt if "k_engine" in r["Kernel_Name"])
    if len(eng) <= a.warmup:
        raise SystemExit("no timed engine launches in the trace")
    t0, t1 = eng[a.warmup][0], max(e for _, e in eng[a.warmup:])
    # runtime shader kernels: copies (hipMemcpy* run as __amd_rocclr_copyBuffer*) and fills (hipMemset*,
    # __amd_rocclr_fillBuffer*: a context's zeroing at creation)
    blits = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kt if "copyBuffer" in r["Kernel_Name"]]
    fills = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kt if "fillBuffer" in r["Kernel_Name"]]
    mc = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "")) for r in
          rows(a.dir, "*memory_copy_trace.csv")]

    def summ(xs):
        inside = [x for x in xs if t0 <= x[0] <= t1]
        return {"inside_timed": len(inside), "inside_ms": round(sum(x[1] - x[0] for x in inside) / 1e6, 3),
                "whole_run": len(xs), "whole_ms": round(sum(x[1] - x[0] for x in xs) / 1e6, 3)}

    out = {"timed_region_ms": round((t1 - t0) / 1e6, 3), "engine_launches_timed": len(eng) - a.warmup,
           "blit_kernels": summ(blits), "fill_kernels": summ(fills), "sdma_copies": summ(mc),
           "sdma_directions_inside": sorted({x[2] for x in mc if t0 <= x[0] <= t1})}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
