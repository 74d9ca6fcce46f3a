"""bench.py host logic that needs no GPU: the N-rank watchdog (a stalled phase ends the rank
with status 3 and names the phase) and the driver's line (size, keys, sidecar)."""
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


def _line(res, detail="gpurun_out/bench_detail_n1.json"):
    import json
    sys.path.insert(0, str(ROOT))
    import bench
    line = bench.compact_line(res, detail)
    text = json.dumps(line)
    assert len(text) <= bench.LINE_MAX_BYTES
    return bench, json.loads(text)


def test_compact_line_fits_and_keeps_the_contract():
    """round 5's 20.9 KB line went unparsed by the driver. The line built
    from that very result (profiles/r05_final_bench_default.json) stays <= 8 KB, parses and
    carries the contract's keys, the roofline / cpu_baseline keys and the sub-summaries."""
    import json
    res = json.loads((ROOT / "profiles" / "r05_final_bench_default.json").read_text())
    assert len(json.dumps(res)) > 20_000
    bench, line = _line(res)
    for k in bench.REQUIRED_KEYS:
        assert k in line, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_stale"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    assert line["value"] == res["value"] and line["ms_per_step"] == res["ms_per_step"]
    for k in ("north_star", "cfg3", "cfg4"):
        assert {"value", "ms", "frac"} <= set(line[k]), k
    assert line["north_star"]["target_met"] is False
    assert line["train_gcn_cfg2"]["step_ms"] > 0 and line["train_gat_cfg3"]["step_ms"] > 0
    assert line["detail"].endswith(".json")


def test_compact_line_n_ranks_and_oversized_fields():
    """The N-rank line (what SCALE parses) keeps the phase maxima; absurdly long strings in any
    sub-object never push the line past the limit."""
    import copy
    import json
    res = json.loads((ROOT / "profiles" / "r03ae_rehearse2_gloo_cfg2.json").read_text())
    res["cpu_baseline"] = {"value": None, "error": "x" * 50_000}
    bench, line = _line(res, "gpurun_out/bench_detail_n2.json")
    assert line["n_gpus"] == 2 and line["phases_ms_max"]["total_ms"] > 0
    assert "row_bounds" not in line
    big = json.loads((ROOT / "profiles" / "r05_final_bench_default.json").read_text())
    for k in ("north_star", "cfg3", "cfg4"):
        big[k]["config"]["workload"] = "w" * 3000
        big[k]["aggregate_ms"] = {str(i): 1.0 for i in range(300)}
    big["roofline"]["kernel"] = "k" * 10_000
    bench, line = _line(copy.deepcopy(big))
    assert "roofline" in line and "cpu_baseline" in line


def test_write_detail_sidecar(tmp_path, monkeypatch):
    import json
    sys.path.insert(0, str(ROOT))
    import bench
    monkeypatch.setenv("GNN_BENCH_DETAIL", str(tmp_path / "d.json"))
    name = bench.write_detail({"value": 1.0, "big": list(range(10))}, 1)
    assert json.loads(Path(name).read_text())["big"][-1] == 9
