"""Price the GAT training block in the degree order: the cfg3 8-head block
(forward + loss.backward(), W / a_src / a_dst requiring grad) on the natural-order graph A
against the same block on P A P^T (nodes relabelled once by degree, graph.degree_order
rows=True; X and dy permuted outside the timing), with each row's neighbours either in the
renamed CSR order or re-sorted ascending. Interleaved in one process, HIP events; per-pass
backward times from ops.gat_backward(timings=...).

    python tools/gat_order_ab.py [--reps 10] [--drop 0.0] [--sparse]
"""
from __future__ import annotations

import argparse
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--drop", type=float, default=0.0)
    ap.add_argument("--sparse", action="store_true")
    a = ap.parse_args()
    import bench
    from graphneuralnetwork_amd import gat as gat_mod
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import CsrGraph, degree_order
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, H, fh, Fin = 1_000_000, 8, 8, 64
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    o = degree_order(g, rows=True)
    g2 = CsrGraph(o.graph.rowptr, o.graph.col, o.graph.val, n, n, symmetric=True)
    rows = torch.repeat_interleave(torch.arange(n, device=dev), g2.rowptr[1:] - g2.rowptr[:-1])
    key, srt = torch.sort(rows * n + g2.col.to(torch.int64))
    g3 = CsrGraph(g2.rowptr, (key % n).to(torch.int32).contiguous(), g2.val[srt].contiguous(),
                  n, n, symmetric=True)
    del rows, key, srt
    torch.manual_seed(0)
    net = getattr(gat_mod, "SpGAT" if a.sparse else "GAT")(Fin, fh, 3, a.drop, 0.2, H).to(dev)
    net.train()
    gen = torch.Generator(dev).manual_seed(3)
    X = torch.randn(n, Fin, device=dev, generator=gen)
    gy = torch.randn(n, H * fh, device=dev, generator=gen)
    X2, gy2 = o.permute_rows(X), o.permute_rows(gy)
    cases = {"natural A": (g, X, gy), "P A P^T (renamed rows)": (g2, X2, gy2),
             "P A P^T (sorted rows)": (g3, X2, gy2)}
    res = {k: {"step": [], "fwd": [], "bwd": []} for k in cases}

    def step(gr, x, y):
        net.zero_grad(set_to_none=True)
        net._heads(x, gr).backward(y)

    for rep in range(a.reps):
        for k, (gr, x, y) in cases.items():
            res[k]["step"] += bench.time_steps(lambda: step(gr, x, y), 3, 1, dev)[0]
            res[k]["fwd"] += bench.time_steps(lambda: net._heads(x, gr), 3, 1, dev)[0]
    # per-pass backward times of the raw ops
    W = torch.cat([m.W for m in net.attentions], 1).detach()
    a_s = torch.cat([m._a_parts()[0] for m in net.attentions]).detach()
    a_d = torch.cat([m._a_parts()[1] for m in net.attentions]).detach()
    mode = ops.GAT_SPARSE if a.sparse else ops.GAT_DENSE
    for k, (gr, x, y) in cases.items():
        wh = torch.mm(x, W)
        el, er = ops.gat_logits(wh, H, fh, a_s, a_d)
        st = torch.empty((n, H), device=dev)
        out = ops.gat_aggregate(gr, wh, el, er, H, fh, 0.2, mode, "elu", dropout_p=a.drop,
                                seed=7, stats=st, a_dst=a_d)
        per = {}
        for i in range(a.reps + 2):
            tl = []
            ops.gat_backward(gr, wh, el, er, st, out, y, a_s, a_d, H, fh, 0.2, mode, True,
                             a.drop, 7, timings=tl)
            torch.cuda.synchronize(dev)
            if i >= 2:
                for name, e0, e1 in tl:
                    per.setdefault(name, []).append(e0.elapsed_time(e1))
        agg = bench.time_steps(lambda: ops.gat_aggregate(gr, wh, el, er, H, fh, 0.2, mode, "elu",
                                                         dropout_p=a.drop, seed=7, stats=st,
                                                         a_dst=a_d), 10, 2, dev)[0]
        print(f"{k}: step {statistics.median(res[k]['step']):.3f} ms, forward "
              f"{statistics.median(res[k]['fwd']):.3f} ms, aggregation (stats) "
              f"{statistics.median(agg):.3f} ms, backward passes "
              + ", ".join(f"{p} {statistics.median(v):.3f}" for p, v in per.items()), flush=True)


if __name__ == "__main__":
    main()
