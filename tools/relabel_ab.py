"""A/B of the degree-ordered graph (graph.degree_order) against the natural R-MAT order, in
one process: the default SpMM on A, the same on A' = P A P^T with X' = P X (hub rows read in
place, no staging copy: XcdHubPlan.direct), and A' with the staging copy kept
(ops.XCD_DIRECT = False). Outputs are compared (Y' = P Y) before timing.

    python tools/relabel_ab.py [--workload cfg2|ns] [--feat 128] [--rounds 5]
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--ks", default="", help="extra in-place variants with K hub rows, e.g. "
                    "131072,524288 (ops.XCD_HUB_ROWS / XCD_HUB_BYTES)")
    ap.add_argument("--degs", default="", help="extra in-place variants with rows of >= D "
                    "edges sliced (ops.XCD_MIN_DEG)")
    a = ap.parse_args()
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import degree_order
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n, e = {"cfg2": (1_000_000, 10_000_000), "ns": (10_000_000, 100_000_000)}[a.workload]
    dev = torch.device("cuda:0")
    s, d = rmat_edges(n, e, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    order = degree_order(g)
    torch.cuda.synchronize()
    t_order = time.perf_counter() - t0
    gp = order.graph
    gc = degree_order(g, rows=False).graph
    F = a.feat
    X = torch.randn(n, F, device=dev)
    b = torch.randn(F, device=dev)
    Xp = order.permute_rows(X)
    Y = torch.empty(n, F, device=dev)
    ref = ops.spmm_forward(g, X, b).clone()
    refp = ref[order.perm]
    variants = {"natural order": (g, X, True), "degree order, in place": (gp, Xp, True),
                "degree order, staged copy": (gp, Xp, False),
                "degree-ordered columns only, in place": (gc, Xp, True)}
    knobs = {}
    k0, d0 = ops.XCD_HUB_ROWS, ops.XCD_MIN_DEG
    for k in (int(v) for v in a.ks.split(",") if v):
        variants[f"degree order, in place, K={k}"] = (gp, Xp, True)
        knobs[f"degree order, in place, K={k}"] = (k, d0)
    for dg in (int(v) for v in a.degs.split(",") if v):
        variants[f"degree order, in place, deg>={dg}"] = (gp, Xp, True)
        knobs[f"degree order, in place, deg>={dg}"] = (k0, dg)

    def run(v):
        gg, xx, direct = variants[v]
        ops.XCD_DIRECT = direct
        k, dg = knobs.get(v, (k0, d0))
        ops.XCD_HUB_ROWS, ops.XCD_HUB_BYTES, ops.XCD_MIN_DEG = k, k * 4 * F, dg
        return ops.spmm_forward(gg, xx, b, out=Y)

    res = {}
    for v in variants:
        run(v)
        torch.cuda.synchronize()
        want = ref if v in ("natural order", "degree-ordered columns only, in place") else refp
        err = float((Y - want).abs().max() / want.abs().max())
        assert err < 1e-5, (v, err)
        gg = variants[v][0]
        k, dg = knobs.get(v, (k0, d0))
        xp = gg._plans.get(next((key for key in gg._plans
                                 if key[0] == "_xcd" and key[1] == min(k, n) and key[2] == dg),
                                None))
        res[v] = {"err": err, "prefix": bool(xp.prefix) if xp is not None else None,
                  "items": xp.n_items if xp is not None else None, "ms": []}
    print(json.dumps({"workload": a.workload, "n": n, "nnz": g.nnz, "feat": F,
                      "degree_order_s": round(t_order, 3)}), flush=True)
    for _ in range(a.rounds):
        for v in variants:
            for _ in range(3):
                run(v)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(10):
                run(v)
            ev[1].record()
            torch.cuda.synchronize()
            res[v]["ms"].append(ev[0].elapsed_time(ev[1]) / 10)
    for v, r in res.items():
        print(json.dumps({"variant": v, "median_ms": round(statistics.median(r["ms"]), 4),
                          "min_ms": round(min(r["ms"]), 4), "max_rel_err": r["err"],
                          "prefix": r["prefix"], "items": r["items"]}), flush=True)
    ops.XCD_DIRECT = True


if __name__ == "__main__":
    main()
