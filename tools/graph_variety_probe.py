"""SpMM on graphs other than the bench's natural-order R-MAT: the same R-MAT with its node
ids permuted (hubs scattered over X, SURVEY 8(d)'s optional seeded relabelling) and a
uniform random graph of the same size (no hubs). Default hub staging vs none.

    python tools/graph_variety_probe.py [--nodes 1000000] [--edges 10000000] [--feat 128]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=10_000_000)
    ap.add_argument("--feat", type=int, default=128)
    args = ap.parse_args()
    from graphneuralnetwork_amd.ops import spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import permute_ids, rmat_edges
    dev = torch.device("cuda:0")
    n, e, F = args.nodes, args.edges, args.feat
    s0, d0 = rmat_edges(n, e, 0)
    graphs = {"rmat": (s0, d0), "rmat_permuted": permute_ids(s0, d0, n, 1)}
    rng = np.random.default_rng(2)
    graphs["uniform"] = (rng.integers(0, n, e), rng.integers(0, n, e))
    X = torch.randn(n, F, device=dev)
    Y = torch.empty(n, F, device=dev)

    def timed(g, hubs):
        f = lambda: spmm_forward(g, X, out=Y, hubs=hubs)  # noqa: E731
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                f()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / 5)
        return statistics.median(ts)

    for name, (s, d) in graphs.items():
        g = gcn_adjacency(torch.from_numpy(np.asarray(s)).to(dev),
                          torch.from_numpy(np.asarray(d)).to(dev), n, device=dev)
        nbytes = g.nnz * (8 + 4 * F) + n * (8 + 4 * F)
        for hubs in (None, 0):
            ms = timed(g, hubs)
            print(json.dumps({"graph": name, "nnz": g.nnz, "hubs": "default" if hubs is None else 0,
                              "ms": ms, "edges_per_s": g.nnz / ms * 1e3,
                              "algo_frac": nbytes / (ms / 1e3) / 8e12}), flush=True)
        del g


if __name__ == "__main__":
    main()
