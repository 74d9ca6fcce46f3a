"""bench.py host logic that needs no GPU: the N-rank watchdog (a stalled phase ends the rank
with status 3 and names the phase) and the achievable-floor model."""
import subprocess
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent


def test_watchdog_names_the_stalled_phase():
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench.WD = bench.Watchdog(5, True); bench.phase('setup', 30); "
            "bench.phase('all_to_all', 0.5); time.sleep(30); print('not reached')" % str(ROOT))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "WATCHDOG rank 5: phase 'all_to_all'" in r.stderr
    assert "not reached" not in r.stdout


def test_watchdog_quiet_when_phases_progress():
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench.WD = bench.Watchdog(0, True); bench.phase('a', 3); time.sleep(0.2); "
            "bench.phase('b', None); time.sleep(2.5); print('ok')" % str(ROOT))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_floor_model_counts():
    sys.path.insert(0, str(ROOT))
    import bench
    # columns in degree order: hubs 0..1 (k_hub = 2); non-hub gathers 2,2,3,5,5,5 -> 6 gathers of
    # 3 distinct rows -> 3 cold re-reads
    col = torch.tensor([0, 1, 0, 2, 2, 3, 5, 5, 5, 1], dtype=torch.int32)
    f = bench.floor_model(col, 6, 2, 128, 10_000, 1.0)
    assert (f["nonhub_gathers"], f["nonhub_distinct_rows"], f["cold_rereads"]) == (6, 3, 3)
    assert f["hub_gathers"] == 4 and f["hbm_bytes"] == 10_000 + 3 * 512
    assert abs(f["hbm_ms"] - f["hbm_bytes"] / 6.3e12 * 1e3) < 1e-12
    assert abs(f["l2_ms"] - 4 * 512 / 26.6e12 * 1e3) < 1e-12
    assert f["floor_ms"] == max(f["hbm_ms"], f["l2_ms"])
