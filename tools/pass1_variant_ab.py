"""A/B of the pass-1 (items) launch of the direct XCD SpMM (column-degree-ordered cfg2/ns
graph) through gnn_dev_spmm_variant_f32: variant 0 (shipped: U = 4, non-temporal stores),
1 (U = 8), 2 (U = 2), 7 (temporal stores: the partial rows stay cached for pass 2). Times
the whole step (pass 1 + pass 2); outputs compared.

    python tools/pass1_variant_ab.py [--workload cfg2|ns] [--variants 0,1,2,7]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--variants", default="0,1,2,7")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    from graphneuralnetwork_amd import _lib, ops
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n, e = {"cfg2": (1_000_000, 10_000_000), "ns": (10_000_000, 100_000_000)}[a.workload]
    dev = torch.device("cuda:0")
    s, d = rmat_edges(n, e, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    F = 128
    ga = ops.column_order(g, F).graph
    X = torch.randn(n, F, device=dev)
    b = torch.randn(F, device=dev)
    ref = ops.spmm_forward(ga, X, b).clone()
    xp = next(p for k, p in ga._plans.items() if isinstance(k, tuple) and k[0] == "_xcd")
    items, rest = xp.direct()
    lib = _lib.load()
    stream = _lib.stream_handle(dev)
    seg = ops.seg_len_for(F)
    p1 = items.plan(seg)
    tp = rest.task_plan(seg, ops.TASK_MAX_DEG, ops.TASK_COST)
    partial = (torch.empty((tp.base.n_seg, F), device=dev) if tp.base.n_seg else None)
    part = torch.empty((xp.n_pos, F), device=dev)
    Y = torch.empty(n, F, device=dev)

    def step(v):
        _lib.check(lib.gnn_dev_spmm_variant_f32(
            items.rowptr.data_ptr(), items.col.data_ptr(), items.val.data_ptr(), items.n_rows,
            X.data_ptr(), F, F, None, part.data_ptr(), F, p1.seg_len, *p1.args(), None, v,
            stream), "variant")
        ops._spmm_tasks_call(lib, rest, rest.col, tp, X, part, F, b, Y, F, partial, 0, stream,
                             "tasks")

    res = {}
    vs = [int(v) for v in a.variants.split(",")]
    for v in vs:
        step(v)
        torch.cuda.synchronize()
        res[v] = {"err": float((Y - ref).abs().max()), "ms": []}
    for _ in range(a.rounds):
        for v in vs:
            for _ in range(3):
                step(v)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(10):
                step(v)
            ev[1].record()
            torch.cuda.synchronize()
            res[v]["ms"].append(ev[0].elapsed_time(ev[1]) / 10)
    print(json.dumps({"workload": a.workload, **{f"variant {v}": {
        "median_ms": round(statistics.median(r["ms"]), 4), "max_abs_diff": r["err"]}
        for v, r in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
