"""Measurement tooling (CPU): the PMC summary's HBM-bytes and wave-state
arithmetic on synthetic rocprofv3 CSVs, and the rate-distortion PSNR."""
import csv
import importlib.util
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, rel))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _counter_csv(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


ENGINE = "void cairo::k_engine<false>(cairo::EngineArgs)"
CONVERT = "cairo::k_convert_batch(cairo::EngineArgs)"


def test_pmc_summary_hbm_and_wave_states(tmp_path, monkeypatch):
    pmc = _load("pmc_summary", "tools/pmc_summary.py")
    src = tmp_path / "prof"
    # three dispatches per kernel: the first (warm-up) is dropped, median of the rest
    _counter_csv(str(src / "prof_fetch" / "run_counter_collection.csv"),
                 [{"Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": v}
                  for k, v in ((ENGINE, 1), (ENGINE, 100), (ENGINE, 300), (CONVERT, 5), (CONVERT, 10), (CONVERT, 10))])
    _counter_csv(str(src / "prof_write" / "run_counter_collection.csv"),
                 [{"Kernel_Name": k, "Counter_Name": "WRITE_SIZE", "Counter_Value": v}
                  for k, v in ((ENGINE, 0), (ENGINE, 50), (ENGINE, 50), (CONVERT, 1), (CONVERT, 4), (CONVERT, 4))])
    sq = {"SQ_WAVES": 1536, "SQ_WAVE_CYCLES": 1000, "SQ_BUSY_CYCLES": 10, "SQ_WAIT_ANY": 700,
          "SQ_WAIT_INST_ANY": 50, "SQ_ACTIVE_INST_ANY": 250, "SQ_ACTIVE_INST_VALU": 128,
          "SQ_INSTS_VALU": 128, "GRBM_GUI_ACTIVE": 8 * 4}
    rows = []
    for _ in range(2):
        rows += [{"Kernel_Name": ENGINE, "Counter_Name": k, "Counter_Value": v} for k, v in sq.items()]
    _counter_csv(str(src / "prof_sq" / "run_counter_collection.csv"), rows)
    monkeypatch.setattr(pmc, "ROOT", str(tmp_path))
    monkeypatch.setattr(sys, "argv", ["pmc_summary", "--round", "rt", "--config", "cfg", "--src", str(src),
                                      "--batch", "2"])
    pmc.main()
    out = json.load(open(tmp_path / "profiles" / "pmc_cfg.json"))
    # median over dispatches 2..3: fetch 200 KiB (x2 gfx950 correction) + write 50 KiB
    assert out["per_launch_hbm_bytes"]["engine"] == (2 * 200 + 50) * 1024
    assert out["per_frame_hbm_bytes"]["engine"] == (2 * 200 + 50) * 1024 // 2
    ws = out["engine_wave_states"]
    assert abs(ws["waiting_frac"] - 0.7) < 1e-9 and abs(ws["issuing_frac"] - 0.25) < 1e-9
    # VALU quad-cycles x 4 over (GRBM / 8 XCDs) x 1024 SIMDs
    assert abs(ws["valu_issue_frac_of_chip"] - 128 * 4 / (4 * 1024)) < 1e-12


def test_rd_sweep_psnr():
    rd = _load("rd_sweep", "tools/rd_sweep.py")
    a = np.full((8, 8), 100, np.int16)
    assert rd.psnr(a, a) == float("inf")
    b = a + 1  # MSE 1 -> 20 log10(255)
    assert abs(rd.psnr(a, b) - 20 * np.log10(255.0)) < 1e-9
