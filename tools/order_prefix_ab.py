"""A/B in one process: the column-degree order with every column ranked (graph.degree_order)
vs only the hub prefix ranked and the rest in id order (``prefix``), on what the order touches:
the XCD-sliced SpMM over A P^T, the scattered-row transform that writes P (X W^T), and for cfg3
the scattered-row GAT projection plus the aggregation.

    python tools/order_prefix_ab.py --workload cfg2|ns|cfg3     (GPU)
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timed(fn, reps=10, rounds=5):
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
    return round(statistics.median(out), 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--prefix", type=int, default=262144)
    a = ap.parse_args()
    import bench
    from graphneuralnetwork_amd.graph import degree_order
    from graphneuralnetwork_amd.ops import (GAT_DENSE, gat_aggregate, gat_project, gcn_transform,
                                            spmm_forward)
    dev = torch.device("cuda:0")
    wl = bench.WORKLOADS[a.workload]
    g = bench.build_graph(wl["nodes"], wl["edges"], dev, 0, 1)
    orders = {"full": degree_order(g, rows=False),
              "prefix": degree_order(g, rows=False, prefix=a.prefix)}
    assert torch.equal(orders["full"].perm[:a.prefix], orders["prefix"].perm[:a.prefix])
    res = {"workload": a.workload, "prefix": a.prefix}
    n = g.n_rows
    if a.workload == "cfg3":
        H, Fh, Fin = 8, 8, 64
        X = torch.randn(n, Fin, device=dev)
        W = torch.randn(Fin, H * Fh, device=dev) * 0.2
        a_s, a_d = torch.randn(H * Fh, device=dev) * 0.3, torch.randn(H * Fh, device=dev) * 0.3
        out = torch.empty(n, H * Fh, device=dev)
        ref = None
        for name, o in orders.items():
            proj = lambda: gat_project(X, W, H, Fh, a_s, a_d, col_rows=o.inv)  # noqa: E731
            wh, el, er = proj()
            agg = lambda: gat_aggregate(o.graph, wh, el, er, H, Fh, 0.2, GAT_DENSE, "elu",  # noqa
                                        out=out)
            agg()
            if ref is None:
                ref = out.clone()
            res[name] = {"project_ms": timed(proj), "aggregate_ms": timed(agg),
                         "max_abs_diff_vs_full": float((out - ref).abs().max())}
            print(json.dumps({name: res[name]}), flush=True)
    else:
        F = 128
        X = torch.randn(n, F, device=dev)
        W = torch.randn(F, F, device=dev) / F ** 0.5
        S = torch.empty(n, F, device=dev)
        Y = torch.empty(n, F, device=dev)
        bias = torch.randn(F, device=dev)
        ref = None
        for name, o in orders.items():
            tf = lambda: gcn_transform(X, W, out=S, out_rows=o.inv, check_rows=False)  # noqa
            tf()
            sp = lambda: spmm_forward(o.graph, S, bias, out=Y)  # noqa: E731
            sp()
            if ref is None:
                ref = Y.clone()
            res[name] = {"transform_rows_ms": timed(tf), "spmm_ms": timed(sp),
                         "layer_ms": timed(lambda: (tf(), sp())),
                         "max_abs_diff_vs_full": float((Y - ref).abs().max())}
            print(json.dumps({name: res[name]}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
