"""Median per-frame engine LDS counters of tools/attr_valu.sh runs (one
directory per build).  usage: python tools/lds_summary.py gpurun_out/valu_4k_lds [frames per dispatch]"""
import collections
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1]
fpd = int(sys.argv[2]) if len(sys.argv) > 2 else 32
for d in sorted(glob.glob(os.path.join(root, "*/"))):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        if "engine" in r["Kernel_Name"]:
            agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    keys = list(next(iter(agg.values())).keys())
    med = {k: statistics.median(v[k] for v in agg.values()) for k in keys}
    print(os.path.basename(d.rstrip("/")), {k.replace("SQ_", ""): f"{v / fpd / 1e6:.1f}M" for k, v in sorted(med.items())})
