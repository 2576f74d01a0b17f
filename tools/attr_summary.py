"""Summarise tools/attr_traffic.sh: fabric reads per frame of each diagnostic
build and the difference to the default one (attr_base).

A build with CAIRO_ATTR_SKIP bit 0 skips the search-window loads, bit 2 the
row coder's inter-prediction loads; everything else runs the same task shapes,
so base - variant is the read traffic those loads cause after the L2
(TCC_EA0_RDREQ by request size, MI355X_MICROARCH.md §HBM: bytes by size, no
blanket FETCH_SIZE correction).  The requested bytes of each source come from
an accounting build (tools/acct.py); together they give the miss share.
usage: python tools/attr_summary.py --src gpurun_out/attr_4k [--batch 28] [--out profiles/r04/attr_4k.json]
"""
import argparse
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pmc_summary import per_kernel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "attr_4k"))
    ap.add_argument("--batch", type=int, default=28, help="frames per engine launch")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = {"method": __doc__.split("\n\n")[1].replace("\n", " "), "frames_per_launch": a.batch, "builds": {}}
    for d in sorted(glob.glob(os.path.join(a.src, "*", ""))):
        name = os.path.basename(os.path.normpath(d))
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        med = {}
        for cn in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_WRREQ_sum"):
            v = per_kernel(f[0], cn).get("engine")
            if v:
                med[cn] = statistics.median(v)
        rd = 32 * med.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * med.get("TCC_EA0_RDREQ_64B_sum", 0) + \
            128 * med.get("TCC_EA0_RDREQ_128B_sum", 0)
        res["builds"][name] = {"requests_per_launch": med, "read_bytes_per_frame": int(rd / a.batch),
                               "write_requests_per_frame": int(med.get("TCC_EA0_WRREQ_sum", 0) / a.batch)}
    base = res["builds"].get("attr_base")
    if base:
        res["attributed_read_bytes_per_frame"] = {
            k: base["read_bytes_per_frame"] - v["read_bytes_per_frame"] for k, v in res["builds"].items()
            if k != "attr_base"}
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
