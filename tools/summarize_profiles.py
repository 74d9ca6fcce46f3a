"""Summaries of a profile round (tools/profile_round.sh output under gpurun_out/prof/):

  profiles/<round>_<wl>_kernel_stats.csv   rocprofv3 --stats of the workload's bench command
  profiles/traffic_<wl>_F<F>.json          FETCH_SIZE x2 + WRITE_SIZE of its roofline kernel(s)
                                           (tools/pmc_traffic.py rules; what bench.py reads)
  profiles/<round>_summary.json            per-kernel L2 hit rates (TCC_HIT / (HIT + MISS))
                                           and the top kernels by total time

    python tools/summarize_profiles.py <round> [--tag r3] [--src gpurun_out/prof]
"""
import argparse
import csv
import json
import shutil
import statistics
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
# workload -> (feat, roofline kernel(s) as in bench.py, selection)
WORKLOADS = {
    "cfg2": (128, "spmm_csr_kernel+spmm_fixup_kernel", ("steps", 7)),
    "ns": (128, "spmm_csr_kernel+spmm_fixup_kernel", ("steps", 7)),
    "cfg3": (64, "gat_csr_kernel+gat_short_kernel+gat_fixup_kernel", ("median", None)),
    "cfg4": (128, "sage_aggregate_kernel<4, 32, 1, 0, true, 8, false>", ("largest", None)),
}


def rows(path):
    return list(csv.DictReader(open(path)))


def counter(path, name, kernel, how):
    vals = [float(r["Counter_Value"]) for r in rows(path)
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name]
    if not vals:
        raise SystemExit(f"no {name} rows for {kernel!r} in {path}")
    mode, n = how
    if mode == "steps":
        return sum(vals) / n, len(vals)
    if mode == "largest":
        return max(vals), len(vals)
    return statistics.median(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round")
    ap.add_argument("--tag", default="r3")
    ap.add_argument("--src", default=str(ROOT / "gpurun_out" / "prof"))
    a = ap.parse_args()
    src = Path(a.src)
    summary = {}
    for wl, (feat, kernel, how) in WORKLOADS.items():
        base = f"{a.tag}_{wl}"
        stats = next((src / f"{base}_stats").rglob("*kernel_stats.csv"), None)
        fetch = next((src / f"{base}_fetch").rglob("*counter_collection.csv"), None)
        write = next((src / f"{base}_write").rglob("*counter_collection.csv"), None)
        l2 = next((src / f"{base}_l2").rglob("*counter_collection.csv"), None)
        if stats is None:
            print(f"{wl}: no kernel stats under {src}")
            continue
        shutil.copy(stats, ROOT / "profiles" / f"{a.round}_{wl}_kernel_stats.csv")
        s = {}
        st = rows(stats)
        top = sorted(st, key=lambda r: -float(r["TotalDurationNs"]))[:8]
        s["_top_kernels_avg_us"] = {r["Name"][:90]: round(float(r["AverageNs"]) / 1e3, 1)
                                    for r in top}
        if fetch is not None and write is not None:
            fw = [(counter(fetch, "FETCH_SIZE", k, how), counter(write, "WRITE_SIZE", k, how))
                  for k in kernel.split("+")]
            f = sum(x[0][0] for x in fw)
            w = sum(x[1][0] for x in fw)
            tr = {"kernel": kernel, "fetch_kib_raw": f, "write_kib": w,
                  "launches": [[x[0][1] for x in fw], [x[1][1] for x in fw]],
                  "fetch_bytes_corrected": 2 * f * 1024, "write_bytes": w * 1024,
                  "traffic_bytes": (2 * f + w) * 1024,
                  "correction": "FETCH_SIZE x2 (gfx950 wide-read halving), WRITE_SIZE exact; "
                                "KiB->B",
                  "selection": {"steps": f"sum of all launches / {how[1]} steps",
                                "largest": "largest launch",
                                "median": "median launch"}[how[0]],
                  "round": a.round}
            (ROOT / "profiles" / f"traffic_{wl}_F{feat}.json").write_text(
                json.dumps(tr, indent=1) + "\n")
            s["_traffic_bytes_per_step"] = tr["traffic_bytes"]
        if l2 is not None:
            hit, miss = {}, {}
            for r in rows(l2):
                d = hit if r["Counter_Name"].startswith("TCC_HIT") else miss
                d[r["Kernel_Name"]] = d.get(r["Kernel_Name"], 0.0) + float(r["Counter_Value"])
            for k in hit:
                tot = hit[k] + miss.get(k, 0.0)
                if tot:
                    s[k.split("(")[0][:90]] = {"l2_hit_rate": round(hit[k] / tot, 3)}
        summary[wl] = s
        print(wl, json.dumps(s.get("_traffic_bytes_per_step")))
    if summary:
        (ROOT / "profiles" / f"{a.round}_summary.json").write_text(
            json.dumps(summary, indent=1) + "\n")


if __name__ == "__main__":
    main()
