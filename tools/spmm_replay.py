"""Measure the SpMM's ceiling by replaying its own access stream.

The product kernels (ops.spmm_forward over the column-ordered graph A P^T: pass 1 over the
XCD-sliced hub items, pass 2 over the rest as packed tasks) are run on the graph's real plans
with only the gathered row ids rewritten in place, so the schedule, the row classes, the
partial rows, the output writes and every instruction stay the kernel's:
  (a) as built                                -- the bench's step
  (b) every hub gather (hub rank < k, pass 1 and pass 2) redirected to rank % T, a table of
      T rows that fits each XCD's 4 MiB L2    -- the measured floor for the hub gathers
  (c) every hub gather to ONE row (L1 / L2 hits) -- hub gathers at their issue cost
  (d) every gather (hub and non-hub) to rank % T -- no HBM gathers at all: the schedule's
      own cost (CSR, partial rows, output)
Interleaved in one process, HIP events, medians. Not product code: the rewritten ids give
wrong sums (never checked), and the originals are restored before the next variant.

    python tools/spmm_replay.py [--workload cfg2|ns] [--reps 20] [--table-rows 2048]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2", choices=("cfg2", "ns"))
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--table-rows", type=int, default=2048)
    ap.add_argument("--only", default=None,
                    help="one variant (a_as_built, b_hub_to_L2_table, ...): per-kernel traces")
    a = ap.parse_args()
    import bench
    from graphneuralnetwork_amd.graph import XcdHubPlan
    from graphneuralnetwork_amd.ops import column_order, spmm_forward
    dev = torch.device("cuda:0")
    wl = bench.WORKLOADS[a.workload]
    F = 128
    g = bench.build_graph(wl["nodes"], wl["edges"], dev, 0, 1)
    order = column_order(g, F)
    ga = order.graph
    gen = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(g.n_cols, F, device=dev, generator=gen)
    b = torch.randn(F, device=dev, generator=gen)
    Y = torch.empty(g.n_rows, F, device=dev)
    spmm_forward(ga, X, b, out=Y)  # builds the plans
    xps = [p for p in ga._plans.values() if isinstance(p, XcdHubPlan)]
    assert len(xps) == 1, "expected one XCD hub plan"
    xp = xps[0]
    items, rest = xp.direct()
    k, T = xp.k, a.table_rows
    i0, r0 = items.col.clone(), rest.col.clone()
    hub_rest = (r0 >= 0) & (r0 < k)
    counts = {"hub_rows_k": k, "table_rows_T": T, "pass1_hub_gathers": int(i0.numel()),
              "pass2_hub_gathers": int(hub_rest.sum()),
              "pass2_nonhub_gathers": int(((r0 >= k)).sum()),
              "pass2_partial_refs": int((r0 < 0).sum()), "nnz": g.nnz}
    print(json.dumps(counts), flush=True)
    variants = {
        "a_as_built": (i0, r0),
        "b_hub_to_L2_table": (i0 % T, torch.where(hub_rest, r0 % T, r0)),
        "c_hub_to_one_row": (torch.zeros_like(i0), torch.where(hub_rest, torch.zeros_like(r0),
                                                                r0)),
        "d_all_to_L2_table": (i0 % T, torch.where(r0 >= 0, r0 % T, r0)),
    }
    if a.only:
        variants = {a.only: variants[a.only]}
    times = {v: [] for v in variants}
    for _ in range(a.reps):
        for v, (ic, rc) in variants.items():
            items.col.copy_(ic)
            rest.col.copy_(rc)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            spmm_forward(ga, X, b, out=Y)  # one untimed launch in the variant's state
            e0.record()
            spmm_forward(ga, X, b, out=Y)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
    items.col.copy_(i0)
    rest.col.copy_(r0)
    comp = bench.compulsory_bytes(g.nnz, g.n_rows, g.n_cols, F)
    res = {v: {"median_ms": round(statistics.median(t), 4), "min_ms": round(min(t), 4),
               "compulsory_frac": round(comp / (statistics.median(t) / 1e3) / 8e12, 4)}
           for v, t in times.items()}
    if "a_as_built" in res and "b_hub_to_L2_table" in res:
        res["a_over_b"] = round(res["a_as_built"]["median_ms"] /
                                res["b_hub_to_L2_table"]["median_ms"], 3)
    res["workload"] = a.workload
    res.update(counts)
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
