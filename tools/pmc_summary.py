"""Summarise rocprofv3 runs of bench.py into profiles/.

Inputs (gpurun_out/, written by the rocprofv3 commands in DESIGN.md §Measurement):
  prof_kt/run_kernel_stats.csv          --kernel-trace --stats
  prof_fetch/run_counter_collection.csv --pmc FETCH_SIZE  (own pass)
  prof_write/run_counter_collection.csv --pmc WRITE_SIZE  (own pass)
  prof_sq/run_counter_collection.csv    --pmc SQ_* + GRBM_GUI_ACTIVE (wave states, optional)
  prof_hit/run_counter_collection.csv   --pmc TCC_HIT/MISS/READ/WRITE_sum (L2 hit rate, optional)
  prof_lds/run_counter_collection.csv   --pmc SQ_LDS_* + SQ_INSTS_LDS (LDS use and conflicts, optional)

Outputs:
  profiles/<round>_<config>_kernel_stats.csv  (copy of the stats summary)
  profiles/pmc_<config>.json                  per-launch HBM bytes per kernel

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE counts half the bytes of
wide streaming reads, so it is doubled; WRITE_SIZE is taken as is.  The median
over the P-frame dispatches is reported (the first frame is intra-only).
The kernel trace gives the engine's busy time per frame (union of the timed
launches' intervals / frames) and the roofline fraction it implies, the same
computation bench.py makes from HIP events.
usage: python tools/pmc_summary.py --round r02 --config 4k [--src gpurun_out/prof_4k]
"""
import argparse
import csv
import json
import os
import shutil
import sys
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHORT = {"k_convert_batch": "convert", "k_engine": "engine"}


def per_kernel(path, counter=None):
    vals = {}
    for r in csv.DictReader(open(path)):
        if counter and r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"]
        for k, short in SHORT.items():
            if f"::{k}(" in name or f"::{k}<false>(" in name:
                vals.setdefault(short, []).append(float(r["Counter_Value"]))
    # drop the first dispatch of each kernel (warm-up: intra frame, cold caches)
    return {k: v[1:] if len(v) > 1 else v for k, v in vals.items()}


SQ = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
      "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE"]


def wave_states(path):
    """Engine wave-state breakdown from one SQ pass (MI355X_MICROARCH.md §PMC:
    WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES, quad-cycles).
    valu_issue_frac: VALU quad-cycles x 4 over the SIMD-cycles of the dispatch
    (GRBM_GUI_ACTIVE summed over 8 XCDs -> per-XCD cycles; 256 CUs x 4 SIMDs)."""
    if not os.path.exists(path):
        return None
    med = {}
    for c in SQ:
        v = per_kernel(path, c).get("engine")
        if v:
            med[c] = statistics.median(v)
    if "SQ_WAVE_CYCLES" not in med:
        return None
    wc = med["SQ_WAVE_CYCLES"]
    out = {"median_per_dispatch": med,
           "waiting_frac": med.get("SQ_WAIT_ANY", 0) / wc,
           "issue_stalled_frac": med.get("SQ_WAIT_INST_ANY", 0) / wc,
           "issuing_frac": med.get("SQ_ACTIVE_INST_ANY", 0) / wc,
           "valu_frac_of_wave_time": med.get("SQ_ACTIVE_INST_VALU", 0) / wc}
    if "GRBM_GUI_ACTIVE" in med:
        cycles = med["GRBM_GUI_ACTIVE"] / 8.0
        out["valu_issue_frac_of_chip"] = med.get("SQ_ACTIVE_INST_VALU", 0) * 4.0 / (cycles * 256 * 4)
    return out


def union_ns(iv):
    """Length of the union of sorted [start, end) intervals."""
    total, s0, e0 = 0, None, None
    for s, e in iv:
        if e0 is None or s > e0:
            if e0 is not None:
                total += e0 - s0
            s0, e0 = s, e
        else:
            e0 = max(e0, e)
    return total + (e0 - s0 if e0 is not None else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r01")
    ap.add_argument("--config", default="720p")
    ap.add_argument("--content", default="band4", help="bench.py --content of the profiled run")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--steps", type=int, default=20, help="timed launches of the profiled bench.py run")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per engine launch in the profiled run (0: the library default for --config)")
    a = ap.parse_args()
    if a.batch <= 0:
        sys.path.insert(0, ROOT)
        import cairo_amd
        from bench import CONFIGS

        w, h = CONFIGS[a.config][:2]
        a.batch = cairo_amd.default_batch(w, h)
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    sfx = "" if a.content == "band4" else f"_{a.content}"
    stats = os.path.join(a.src, "prof_kt", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out_dir, f"{a.round}_{a.config}{sfx}_kernel_stats.csv"))
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
    trace = os.path.join(a.src, "prof_kt", "run_kernel_trace.csv")
    if os.path.exists(trace):  # the same figures as bench.py's roofline, from the dispatch timestamps
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(trace))
                    if "::k_engine<false>(" in r["Kernel_Name"])
        timed = iv[-a.steps:]  # bench.py's timed launches follow the warm-up ones (ctx.sync between)
        if timed:
            busy = union_ns(timed) / 1e6
            res["engine_timed_launches"] = len(timed)
            res["engine_avg_launch_ms_rocprof"] = round(statistics.mean(e - s for s, e in timed) / 1e6, 3)
            res["engine_busy_ms_per_frame_rocprof"] = round(busy / (len(timed) * a.batch), 4)
            sys.path.insert(0, ROOT)
            from bench import CONFIGS, HBM_PEAK_GBS, algorithmic_bytes

            w, h, ring = CONFIGS[a.config][:3]
            ab = algorithmic_bytes(w, h, ring)["engine"]
            res["roofline_frac_rocprof"] = round(ab / (res["engine_busy_ms_per_frame_rocprof"] * 1e-3) / 1e9 /
                                                 HBM_PEAK_GBS, 6)
    log = os.path.join(a.src, "prof_kt.log")
    if os.path.exists(log):  # bench.py's own HIP-event figures in the traced run (must agree with the trace)
        lines = [ln for ln in open(log) if ln.startswith('{"metric"')]
        if lines:
            b = json.loads(lines[-1])
            res["bench_under_trace"] = {"value": b["value"], "ms_per_step": b["ms_per_step"],
                                        "engine_busy_ms_per_frame": b["roofline"]["engine_busy_ms_per_frame"],
                                        "avg_launch_ms": b["roofline"]["avg_launch_ms"],
                                        "frac": b["roofline"]["frac"]}
    # read requests by size (TCC_EA0_RDREQ_32B / 64B / 128B) and the uncached
    # 32-byte ones (agent-scope hand-off polls and granule loads): bytes by
    # request size, no blanket FETCH_SIZE correction
    rs = os.path.join(a.src, "prof_rdsize", "run_counter_collection.csv")
    rq = os.path.join(a.src, "prof_req", "run_counter_collection.csv")
    if os.path.exists(rs):
        med = {}
        for cn in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum",
                   "TCC_EA0_RD_UNCACHED_32B_sum"):
            v = per_kernel(rs, cn).get("engine")
            if v:
                med[cn] = statistics.median(v)
        if os.path.exists(rq):
            for cn in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"):
                v = per_kernel(rq, cn).get("engine")
                if v:
                    med[cn] = statistics.median(v)
        if med:
            n32, n64, n128 = (med.get(f"TCC_EA0_RDREQ_{k}_sum", 0) for k in ("32B", "64B", "128B"))
            rd = 32 * n32 + 64 * n64 + 128 * n128
            wr = (64 * med["TCC_EA0_WRREQ_64B_sum"] + 32 * (med["TCC_EA0_WRREQ_sum"] - med["TCC_EA0_WRREQ_64B_sum"])
                  if "TCC_EA0_WRREQ_sum" in med else None)
            res["engine_requests_per_launch"] = med
            res["engine_read_bytes_by_size_per_frame"] = int(rd / a.batch)
            res["engine_read_uncached_32b_share"] = round(med.get("TCC_EA0_RD_UNCACHED_32B_sum", 0) /
                                                          max(n32 + n64 + n128, 1), 4)
            if wr is not None:
                res["engine_write_bytes_by_size_per_frame"] = int(wr / a.batch)
                res["per_frame_hbm_bytes_sized"] = int((rd + wr) / a.batch)
            if "TCC_EA0_RDREQ_DRAM_sum" in med and "TCC_EA0_RDREQ_sum" in med:
                res["engine_read_requests_dram_share"] = round(med["TCC_EA0_RDREQ_DRAM_sum"] /
                                                               max(med["TCC_EA0_RDREQ_sum"], 1), 4)
    # L2 hits / misses (one pass): how much of the requested traffic the XCD L2s absorb
    hp = os.path.join(a.src, "prof_hit", "run_counter_collection.csv")
    if os.path.exists(hp):
        med = {}
        for cn in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_READ_sum", "TCC_WRITE_sum"):
            v = per_kernel(hp, cn).get("engine")
            if v:
                med[cn] = statistics.median(v)
        if med:
            hit, miss = med.get("TCC_HIT_sum", 0), med.get("TCC_MISS_sum", 0)
            res["engine_l2"] = {"median_per_dispatch": med,
                                "hit_rate": round(hit / max(hit + miss, 1), 4),
                                "reads_per_frame": int(med.get("TCC_READ_sum", 0) / a.batch),
                                "writes_per_frame": int(med.get("TCC_WRITE_sum", 0) / a.batch)}
    # LDS (one pass): indexed-access cycles per CU against the dispatch's
    # cycles, and the share of them spent on bank conflicts / unaligned stalls
    lp = os.path.join(a.src, "prof_lds", "run_counter_collection.csv")
    if os.path.exists(lp):
        med = {}
        for cn in ("SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_UNALIGNED_STALL",
                   "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"):
            v = per_kernel(lp, cn).get("engine")
            if v:
                med[cn] = statistics.median(v)
        if "SQ_LDS_IDX_ACTIVE" in med and "GRBM_GUI_ACTIVE" in med:
            idx = med["SQ_LDS_IDX_ACTIVE"]
            res["engine_lds"] = {"median_per_dispatch": med,
                                 "lds_busy_frac_per_cu": round(idx / 256 / (med["GRBM_GUI_ACTIVE"] / 8.0), 4),
                                 "bank_conflict_share": round(med.get("SQ_LDS_BANK_CONFLICT", 0) / max(idx, 1), 4),
                                 "unaligned_stall_share": round(med.get("SQ_LDS_UNALIGNED_STALL", 0) / max(idx, 1), 4),
                                 "lds_issue_stall_frac_of_wave_time":
                                     round(med.get("SQ_WAIT_INST_LDS", 0) / max(med.get("SQ_WAVE_CYCLES", 1), 1), 4)}
    ws = wave_states(os.path.join(a.src, "prof_sq", "run_counter_collection.csv"))
    if ws:
        res["engine_wave_states"] = ws
    path = os.path.join(out_dir, f"pmc_{a.config}{sfx}.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res["per_launch_hbm_bytes"]))


if __name__ == "__main__":
    main()
