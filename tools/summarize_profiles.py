"""Summaries of a profile round (tools/profile_round.sh output under gpurun_out/prof/):

  profiles/<round>_<wl>_kernel_stats.csv   rocprofv3 --stats of the workload's bench command
  profiles/traffic_<wl>_F<F>.json          FETCH_SIZE x2 + WRITE_SIZE of its roofline kernel(s)
                                           (tools/pmc_traffic.py rules; what bench.py reads),
                                           stamped with the source tree it was measured on
  profiles/<round>_summary.json            per workload: the top kernels by total time, every
                                           kernel's L2 hit rate (TCC_HIT / (HIT + MISS)), and
                                           per roofline-kernel INSTANCE (pass 1, pass 2, fix-up
                                           of the XCD-sliced SpMM are template instances of one
                                           name) the average duration, the corrected FETCH /
                                           WRITE bytes per step, the L2 hit rate and, when the
                                           round has an SQ pass, the wave-cycle split

    python tools/summarize_profiles.py <round> [--tag r5] [--src gpurun_out/prof]

The stamp is read from <src>/<tag>_stamp.txt (bench.source_stamp() written on the GPU box by
tools/profile_round.sh before the passes); without it the summary says "unstamped".
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
    "cfg3": (64, "gat_eh_kernel+gat_csr_kernel+gat_short_kernel+gat_task_kernel+gat_fixup_kernel",
             ("median", None)),
    "cfg4": (128, "sage_aggregate_kernel<4, 32, 1, 0, true, 8, false>", ("largest", None)),
}
SQ = ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU",
      "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_WAVES")


def rows(path):
    return list(csv.DictReader(open(path)))


def counter(path, name, kernel, how):
    vals = [float(r["Counter_Value"]) for r in rows(path)
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name]
    if not vals:  # a kernel of the list this schedule does not launch
        print(f"  (no {name} rows for {kernel!r})")
        return 0.0, 0
    mode, n = how
    if mode == "steps":
        return sum(vals) / n, len(vals)
    if mode == "largest":
        return max(vals), len(vals)
    return statistics.median(vals), len(vals)


def by_instance(path, kernels):
    """{instance name: {counter: [values per launch]}} for the launches of the roofline kernels."""
    out = {}
    for r in rows(path):
        name = r["Kernel_Name"]
        if any(k in name for k in kernels):
            out.setdefault(name.split("(")[0], {}).setdefault(r["Counter_Name"], []).append(
                float(r["Counter_Value"]))
    return out


def instance_table(stats, fetch, write, l2, sq, kernels, how):
    """Per roofline-kernel instance, per step (steps selection) or per launch (median/largest)."""
    def agg(vals):
        mode, n = how
        if mode == "steps":
            return sum(vals) / n
        return max(vals) if mode == "largest" else statistics.median(vals)

    table = {}
    if stats is not None:
        for r in rows(stats):
            name = r["Name"].split("(")[0]
            if any(k in name for k in kernels):
                table.setdefault(name, {})["avg_us"] = round(float(r["AverageNs"]) / 1e3, 2)
                table[name]["launches"] = int(r["Calls"])
    for path, key, scale in ((fetch, "fetch_bytes", 2 * 1024), (write, "write_bytes", 1024)):
        if path is None:
            continue
        for name, c in by_instance(path, kernels).items():
            v = c.get("FETCH_SIZE" if key == "fetch_bytes" else "WRITE_SIZE")
            if v:
                table.setdefault(name, {})[key] = agg(v) * scale
    if l2 is not None:
        for name, c in by_instance(l2, kernels).items():
            hit = sum(v for k, vs in c.items() if k.startswith("TCC_HIT") for v in vs)
            miss = sum(v for k, vs in c.items() if k.startswith("TCC_MISS") for v in vs)
            if hit + miss:
                table.setdefault(name, {})["l2_hit_rate"] = round(hit / (hit + miss), 3)
    if sq is not None:
        for name, c in by_instance(sq, kernels).items():
            wc = sum(c.get("SQ_WAVE_CYCLES", []))
            e = table.setdefault(name, {})
            if wc:
                for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                    if k in c:
                        e[k.lower().replace("sq_", "") + "_frac"] = round(sum(c[k]) / wc, 3)
            waves = sum(c.get("SQ_WAVES", []))
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU"):
                if k in c:
                    e[k.lower() + "_per_launch"] = statistics.mean(c[k])
                    if waves:
                        e[k.lower() + "_per_wave"] = round(sum(c[k]) / waves, 1)
            if waves:
                e["waves_per_launch"] = waves / len(c["SQ_WAVES"])
    for e in table.values():
        if "fetch_bytes" in e and "write_bytes" in e:
            e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
    return table


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round")
    ap.add_argument("--tag", default="r5")
    ap.add_argument("--src", default=str(ROOT / "gpurun_out" / "prof"))
    ap.add_argument("--workloads", default=",".join(WORKLOADS))
    a = ap.parse_args()
    src = Path(a.src)
    stamp_file = src / f"{a.tag}_stamp.txt"
    stamp = stamp_file.read_text().strip() if stamp_file.exists() else None
    summary = {"_source_stamp": stamp or "unstamped"}
    for wl in a.workloads.split(","):
        feat, kernel, how = WORKLOADS[wl]
        base = f"{a.tag}_{wl}"

        def find(kind, pat):
            d = src / f"{base}_{kind}"
            return next(d.rglob(pat), None) if d.exists() else None
        stats = find("stats", "*kernel_stats.csv")
        fetch = find("fetch", "*counter_collection.csv")
        write = find("write", "*counter_collection.csv")
        l2 = find("l2", "*counter_collection.csv")
        sq = find("sq", "*counter_collection.csv")
        if stats is None:
            print(f"{wl}: no kernel stats under {src}")
            continue
        shutil.copy(stats, ROOT / "profiles" / f"{a.round}_{wl}_kernel_stats.csv")
        s = {}
        st = rows(stats)
        top = sorted(st, key=lambda r: -float(r["TotalDurationNs"]))[:8]
        s["_top_kernels_avg_us"] = {r["Name"][:90]: round(float(r["AverageNs"]) / 1e3, 1)
                                    for r in top}
        parts = kernel.split("+")
        s["_roofline_kernel_instances"] = instance_table(stats, fetch, write, l2, sq, parts, how)
        s["_instance_selection"] = {"steps": f"sum of all launches / {how[1]} steps",
                                    "largest": "largest launch", "median": "median launch"}[how[0]]
        if fetch is not None and write is not None:
            fw = [(counter(fetch, "FETCH_SIZE", k, how), counter(write, "WRITE_SIZE", k, how))
                  for k in parts]
            f = sum(x[0][0] for x in fw)
            w = sum(x[1][0] for x in fw)
            tr = {"kernel": kernel, "fetch_kib_raw": f, "write_kib": w,
                  "launches": [[x[0][1] for x in fw], [x[1][1] for x in fw]],
                  "fetch_bytes_corrected": 2 * f * 1024, "write_bytes": w * 1024,
                  "traffic_bytes": (2 * f + w) * 1024,
                  "correction": "FETCH_SIZE x2 (gfx950 wide-read halving), WRITE_SIZE exact; "
                                "KiB->B",
                  "selection": s["_instance_selection"],
                  "round": a.round, "source_stamp": stamp,
                  "per_instance": {k: {kk: v[kk] for kk in ("fetch_bytes", "write_bytes",
                                                            "traffic_bytes", "l2_hit_rate",
                                                            "avg_us") if kk in v}
                                   for k, v in s["_roofline_kernel_instances"].items()}}
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
        for k, v in s["_roofline_kernel_instances"].items():
            print("   ", k, json.dumps(v))
    if len(summary) > 1:
        (ROOT / "profiles" / f"{a.round}_summary.json").write_text(
            json.dumps(summary, indent=1) + "\n")


if __name__ == "__main__":
    main()
