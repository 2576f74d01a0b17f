"""Summarise rocprofv3 runs of bench.py into profiles/.

Inputs (gpurun_out/, written by the rocprofv3 commands in DESIGN.md §Measurement):
  prof_kt/run_kernel_stats.csv          --kernel-trace --stats
  prof_fetch/run_counter_collection.csv --pmc FETCH_SIZE  (own pass)
  prof_write/run_counter_collection.csv --pmc WRITE_SIZE  (own pass)

Outputs:
  profiles/<round>_<config>_kernel_stats.csv  (copy of the stats summary)
  profiles/pmc_<config>.json                  per-launch HBM bytes per kernel

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE counts half the bytes of
wide streaming reads, so it is doubled; WRITE_SIZE is taken as is.  The median
over the P-frame dispatches is reported (the first frame is intra-only).
usage: python tools/pmc_summary.py --round r01 --config 720p [--src gpurun_out]
"""
import argparse
import csv
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHORT = {"k_convert_batch": "convert", "k_engine": "engine"}


def per_kernel(path):
    vals = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        for k, short in SHORT.items():
            if f"::{k}(" in name or f"::{k}<false>(" in name:
                vals.setdefault(short, []).append(float(r["Counter_Value"]))
    # drop the first dispatch of each kernel (warm-up: intra frame, cold caches)
    return {k: v[1:] if len(v) > 1 else v for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r01")
    ap.add_argument("--config", default="720p")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--batch", type=int, default=16, help="frames per engine launch in the profiled run")
    a = ap.parse_args()
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    stats = os.path.join(a.src, "prof_kt", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out_dir, f"{a.round}_{a.config}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(a.src, "prof_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(a.src, "prof_write", "run_counter_collection.csv"))
    res = {"config": a.config, "round": a.round,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py; "
                     "KiB per dispatch, median over dispatches after the first; HBM bytes = 2*FETCH_SIZE (gfx950 "
                     "correction, MI355X_MICROARCH.md §HBM) + WRITE_SIZE; per frame = per launch / frames per launch. "
                     "Infinity-Cache hits are counted.",
           "frames_per_launch": a.batch,
           "fetch_kib_raw": {}, "write_kib": {}, "per_launch_hbm_bytes": {}, "per_frame_hbm_bytes": {},
           "dispatches": {}}
    for k in sorted(set(fetch) & set(write)):
        f, w = statistics.median(fetch[k]), statistics.median(write[k])
        res["fetch_kib_raw"][k] = f
        res["write_kib"][k] = w
        res["per_launch_hbm_bytes"][k] = int(round((2 * f + w) * 1024))
        res["per_frame_hbm_bytes"][k] = int(round((2 * f + w) * 1024 / a.batch))
        res["dispatches"][k] = min(len(fetch[k]), len(write[k]))
    path = os.path.join(out_dir, f"pmc_{a.config}.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res["per_launch_hbm_bytes"]))


if __name__ == "__main__":
    main()
