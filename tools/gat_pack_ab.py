"""A/B in one process at cfg3 (1M / 20M nnz, 8 heads x 8): the GAT aggregation reading Wh and
er from separate tables vs one packed [Wh | er | el] row (gat_project packed=True), natural
column order with the hub staging, and the column-degree order (hub rows in place; packed
[Wh | er] rows scattered, el beside them).

    python tools/gat_pack_ab.py
"""
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
    return out


def main():
    from graphneuralnetwork_amd.ops import GAT_DENSE, gat_aggregate, gat_column_order, gat_project
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, H, fh, k = 1_000_000, 8, 8, 64
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    x = torch.randn(n, k, device=dev)
    w = torch.randn(k, H * fh, device=dev) * 0.2
    a_s, a_d = torch.randn(H * fh, device=dev) * 0.3, torch.randn(H * fh, device=dev) * 0.3
    order = gat_column_order(g, H, fh)
    p_sep = gat_project(x, w, H, fh, a_s, a_d)
    p_pack = gat_project(x, w, H, fh, a_s, a_d, packed=True)
    p_ord = gat_project(x, w, H, fh, a_s, a_d, col_rows=order.inv)
    # column order, packed: [Wh | er] rows scattered, el in a same-stride buffer
    buf = torch.empty(n, H * fh + 2 * H, device=dev)
    elb = torch.empty(n, H * fh + 2 * H, device=dev)
    buf[order.inv, :H * fh] = p_sep[0]
    buf[order.inv, H * fh:H * fh + H] = p_sep[2]
    elb[:, :H] = p_sep[1]
    p_ord_pack = (buf[:, :H * fh], elb[:, :H], buf[:, H * fh:H * fh + H])
    out = torch.empty(n, H * fh, device=dev)
    ref = gat_aggregate(g, *p_sep, H, fh, 0.2, GAT_DENSE, "elu").clone()
    var = {"separate": (g, p_sep), "packed": (g, p_pack), "column order separate": (order.graph, p_ord),
           "column order packed": (order.graph, p_ord_pack)}
    res = {v: [] for v in var}
    for v, (gg, p) in var.items():
        gat_aggregate(gg, *p, H, fh, 0.2, GAT_DENSE, "elu", out=out)
        torch.cuda.synchronize()
        err = float((out - ref).abs().max())
        assert err < 1e-5, (v, err)
    for _ in range(3):
        for v, (gg, p) in var.items():
            res[v].extend(timed(lambda: gat_aggregate(gg, *p, H, fh, 0.2, GAT_DENSE, "elu",
                                                      out=out)))
    print(json.dumps({v: round(statistics.median(t), 4) for v, t in res.items()}), flush=True)


if __name__ == "__main__":
    main()
