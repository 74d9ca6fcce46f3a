"""A/B in one process: the GAT projection (cfg3 shape, 1M x 64 -> 8 x 8 heads) in order vs
with Wh / er scattered to col_rows (gat_project col_rows=): a random permutation, the cfg3
graph's column-degree order, and the identity (the scatter path with sequential addresses).

    python tools/project_rows_ab.py
"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timed(fn, reps=20, rounds=5):
    out = []
    for _ in range(rounds):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) / reps)
    return statistics.median(out)


def main():
    from graphneuralnetwork_amd.graph import degree_order
    from graphneuralnetwork_amd.ops import gat_project
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, H, fh, k = 1_000_000, 8, 8, 64
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    inv_deg = degree_order(g, rows=False).inv
    x = torch.randn(n, k, device=dev)
    w = torch.randn(k, H * fh, device=dev) * 0.2
    a_s, a_d = torch.randn(H * fh, device=dev), torch.randn(H * fh, device=dev)
    res = {}
    for name, rows in (("in order", None), ("identity", torch.arange(n, device=dev)),
                       ("degree order inv", inv_deg), ("random", torch.randperm(n, device=dev))):
        res[name] = timed(lambda: gat_project(x, w, H, fh, a_s, a_d, col_rows=rows))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
