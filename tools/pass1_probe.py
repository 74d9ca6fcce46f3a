"""Pass 1 of the XCD-sliced SpMM (items -> partial rows) on the column-degree-ordered cfg2
graph, timed alone: one wave per item (the shipped plain-kernel launch) vs packed row tasks
over the same items (the XCD placement of items is lost there: a rate probe only), each also
with the columns folded into an L2-resident set (col % 4096).

    python tools/pass1_probe.py [--workload cfg2|ns]
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
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    a = ap.parse_args()
    from graphneuralnetwork_amd import _lib, ops
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n, e = {"cfg2": (1_000_000, 10_000_000), "ns": (10_000_000, 100_000_000)}[a.workload]
    dev = torch.device("cuda:0")
    s, d = rmat_edges(n, e, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    F = 128
    order = ops.column_order(g, F)
    ga = order.graph
    X = torch.randn(n, F, device=dev)
    ops.spmm_forward(ga, X)
    xp = next(p for k, p in ga._plans.items() if isinstance(k, tuple) and k[0] == "_xcd")
    items, rest = xp.direct()
    folded = CsrGraph(items.rowptr, (items.col % 4096).contiguous(), items.val, items.n_rows,
                      items.n_cols)
    part = torch.empty((xp.n_pos, F), device=dev)
    lib = _lib.load()
    stream = _lib.stream_handle(dev)
    seg = ops.seg_len_for(F)

    def plain(gr):
        p1 = gr.plan(seg)
        return lambda: _lib.check(lib.gnn_spmm_csr_f32(
            gr.rowptr.data_ptr(), gr.col.data_ptr(), gr.val.data_ptr(), gr.n_rows, X.data_ptr(),
            F, F, None, part.data_ptr(), F, p1.seg_len, *p1.args(), None, 0, stream), "plain")

    def tasks(gr, cost):
        tp = gr.task_plan(seg, 128, cost)
        return lambda: ops._spmm_tasks_call(lib, gr, gr.col, tp, X, None, F, None, part, F, None,
                                            0, stream, "tasks")

    res = {"workload": a.workload, "items": xp.n_items, "positions": xp.n_pos,
           "item_edges": items.nnz}
    for name, gr in (("as built", items), ("folded", folded)):
        res[f"plain {name}"] = timed(plain(gr))
        for cost in (128, 256, 512):
            res[f"tasks{cost} {name}"] = timed(tasks(gr, cost))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
