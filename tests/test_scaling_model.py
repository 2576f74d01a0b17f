"""The partition model behind DESIGN §6 ("Hop latency and the partition
model", tools/scaling_model.py): the committed table is what the model gives
for its recorded inputs, and the model keeps the properties the section reads
off it.  CPU only."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import scaling_model  # noqa: E402


def test_committed_table_reproduces(tmp_path):
    """Re-running the model with the inputs recorded in
    profiles/r06/scaling_model.json gives the same rows."""
    ref = json.load(open(os.path.join(ROOT, "profiles", "r06", "scaling_model.json")))
    i = ref["inputs"]
    out = tmp_path / "m.json"
    cmd = [sys.executable, os.path.join(ROOT, "tools", "scaling_model.py"), "--t1", str(i["t1"]),
           "--lag-idle", str(i["lag_idle"]), "--lag-full", str(i["lag_full"]), "--hop", str(i["hop"]),
           "--hop0", str(i["hop0"]), "--xgmi", i["xgmi"], "--json", str(out)]
    if i.get("coder_full_ms"):
        cmd += ["--coder-full-ms", str(i["coder_full_ms"])]
    subprocess.run(cmd, check=True, capture_output=True)
    got = json.load(open(out))
    assert got["one_gpu_fps"] == ref["one_gpu_fps"]
    assert got["rows"] == ref["rows"]


def test_one_gpu_is_throughput_bound():
    """N = 1: the lag bound (1 / 290 us) is far above one GPU's throughput
    (1 / T1), so F = 1 / T1."""
    f, cap = scaling_model.solve(1, 1.233, 180.0, 290.0, 0.0)
    assert f == pytest.approx(cap, rel=1e-6)
    assert cap == pytest.approx(1e3 / 1.233, rel=1e-9)


@pytest.mark.parametrize("xgmi", [0.0, 2.0, 5.0])
@pytest.mark.parametrize("n", [2, 4, 8])
def test_interleave_never_below_row_shard(n, xgmi):
    """The reading DESIGN §6 takes from the table: with one hop per frame and
    whole frames per GPU, the frame interleave is at least the row shard (two
    hops, the 135-row imbalance) at every N and link latency."""
    import math

    fi, _ = scaling_model.solve(n, 1.233, 180.0, 290.0, 1.98 + xgmi)
    imb = math.ceil(135 / n) * n / 135
    fr, _ = scaling_model.solve(n, 1.233, 180.0, 290.0, (0.74 + xgmi) + (1.98 + xgmi), imb)
    assert fi >= fr


def test_lag_bound_at_eight():
    """At N = 8 both partitions are lag-bound: the rate is 1 / L(u), below
    the throughput bound, and about 5x one GPU."""
    f8, cap8 = scaling_model.solve(8, 1.233, 180.0, 290.0, 1.98)
    f1, _ = scaling_model.solve(1, 1.233, 180.0, 290.0, 0.0)
    assert f8 < 0.999 * cap8
    assert 4.5 < f8 / f1 < 5.5
