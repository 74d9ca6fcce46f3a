"""cfg4 probe: the GraphSAGE [25, 10] forward on the natural-order R-MAT graph and table vs
the same graph and table relabelled by degree (graph.degree_order rows + columns: hub rows
first in the table), the same seeds mapped, each sampled on its own graph. Times the forward
and the layer-0 gather-mean (interleaved rounds).

    python tools/sage_order_probe.py
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
    return out


def main():
    from graphneuralnetwork_amd.graph import degree_order
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.ops import sage_gather_aggregate
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import sample_batch, symmetric_adjacency
    dev = torch.device("cuda:0")
    n, F = 10_000_000, 128
    s, d = rmat_edges(n, 100_000_000, 0)
    adj = symmetric_adjacency(s, d, n, device=dev)
    del s, d
    o = degree_order(adj, rows=True)
    adj2 = o.graph
    gen = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(n, F, device=dev, generator=gen)
    table2 = o.permute_rows(table)
    deg = adj.rowptr[1:] - adj.rowptr[:-1]
    cand = torch.nonzero(deg > 0).view(-1)
    seeds = cand[torch.randperm(cand.numel(), device=dev, generator=gen)[:8192]]
    b1 = sample_batch(adj, seeds, (25, 10), seed=0)
    b2 = sample_batch(adj2, o.inv[seeds], (25, 10), seed=0)
    net = GraphSAGE(2, F, F, False, agg_func="MEAN", Unsupervised=False, class_size=3).to(dev).eval()
    f1, f2 = b1.forward_args(table), b2.forward_args(table2)
    res = {"frontier": [int(b1.frontier.numel()), int(b2.frontier.numel())],
           "fwd": ([], []), "gather0": ([], [])}
    with torch.no_grad():
        for _ in range(3):
            for i, (f, b, t) in enumerate(((f1, b1, table), (f2, b2, table2))):
                res["fwd"][i].extend(timed(lambda: net(*f, None, None, None, None, None)))
                res["gather0"][i].extend(timed(lambda: sage_gather_aggregate(
                    t, b.frontier_nbrs, "MEAN", check=False)))
    out = {"frontier": res["frontier"]}
    for k in ("fwd", "gather0"):
        out[k] = {"natural_ms": round(statistics.median(res[k][0]), 4),
                  "degree_order_ms": round(statistics.median(res[k][1]), 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
