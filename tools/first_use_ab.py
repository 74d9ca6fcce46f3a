"""A/B of the non-hub column order of the column-degree-ordered SpMM.

The hub rows (the K = 256 Ki highest in-degree columns) stay the first K rows of X in every
variant; the other columns follow in
  degree     -- descending in-degree (the shipped order, graph.degree_order)
  id         -- ascending ids (graph.degree_order prefix=K, tail="id")
  first_use  -- the CSR position of their first edge (tail="first_use"): the rows a
                row-ordered pass touches for the first time lie together in memory.
The hub set, items, slices and edge order are the same, so Y is bit-identical; only the
addresses of the non-hub rows move. Interleaved timing in one process.

    python tools/first_use_ab.py [--workload ns|cfg2] [--reps 20]
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
    ap.add_argument("--workload", default="ns", choices=["ns", "cfg2"])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from graphneuralnetwork_amd.graph import degree_order
    from graphneuralnetwork_amd.ops import spmm_forward, xcd_hub_rows_for
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, m = (10_000_000, 100_000_000) if a.workload == "ns" else (1_000_000, 10_000_000)
    F = 128
    s, d = rmat_edges(n, m, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    K = xcd_hub_rows_for(n, F)
    orders = {t: degree_order(g, rows=False, prefix=K, tail=t) for t in ("degree", "id", "first_use")}
    gen = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(n, F, device=dev, generator=gen)   # the support, original ids
    b = torch.randn(F, device=dev, generator=gen)
    Xs = {t: o.permute_rows(X) for t, o in orders.items()}  # row j = old column perm[j]
    Y = torch.empty(n, F, device=dev)
    ref = None
    res = {}
    for rnd in range(3):
        for t, o in orders.items():
            spmm_forward(o.graph, Xs[t], b, out=Y)
            torch.cuda.synchronize()
            if ref is None:
                ref = Y.clone()
            elif rnd == 0:
                assert torch.equal(Y, ref), t
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(a.reps)]
            for e0, e1 in ev:
                e0.record()
                spmm_forward(o.graph, Xs[t], b, out=Y)
                e1.record()
            torch.cuda.synchronize()
            res.setdefault(t, []).extend(e0.elapsed_time(e1) for e0, e1 in ev)
    print(json.dumps({"workload": a.workload, "hub_rows": K,
                      "median_ms": {t: round(statistics.median(v), 4) for t, v in res.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
