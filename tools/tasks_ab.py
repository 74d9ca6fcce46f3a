"""A/B of the packed row tasks (gnn_spmm_csr_tasks_f32) against one wave per short row, inside
one process, on the bench graphs; the outputs are compared too.

    python tools/tasks_ab.py [--workload cfg2|ns] [--feat 128] [--grid "64:256,64:128,..."]
                             [--column-order]
"""
import argparse
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timed(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--grid", default="64:256,64:128,64:512,32:256,128:256,16:256")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--column-order", action="store_true",
                    help="over the column-degree-ordered graph (ops.column_order), as the bench")
    a = ap.parse_args()
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n, e = {"cfg2": (1_000_000, 10_000_000), "ns": (10_000_000, 100_000_000),
            "small": (200_000, 2_000_000)}[a.workload]
    dev = torch.device("cuda:0")
    s, d = rmat_edges(n, e, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    F = a.feat
    if a.column_order:
        g = ops.column_order(g, F).graph
    X = torch.randn(n, F, device=dev)
    b = torch.randn(F, device=dev)
    Y = torch.empty(n, F, device=dev)
    ops.SPMM_TASKS = False
    ref = ops.spmm_forward(g, X, b).clone()
    configs = [None] + [tuple(int(v) for v in c.split(":")) for c in a.grid.split(",") if c]
    res = {c: [] for c in configs}

    def run(c):
        if c is None:
            ops.SPMM_TASKS = False
        else:
            ops.SPMM_TASKS = True
            ops.TASK_MAX_DEG, ops.TASK_COST = c
        return timed(lambda: ops.spmm_forward(g, X, b, out=Y))

    for c in configs:  # plans + correctness
        run(c)
        err = float((Y - ref).abs().max() / ref.abs().max())
        print(f"config {c}: max |diff| / max |ref| = {err:.2e}", flush=True)
        assert err < 1e-5, err
    for r in range(a.rounds):
        for c in configs:
            res[c].append(run(c))
    print(f"workload {a.workload} n={n} nnz={g.nnz} F={F}")
    for c in configs:
        name = "one wave per row" if c is None else f"tasks max_deg={c[0]} cost={c[1]}"
        print(f"  {name:34s} {min(res[c]):8.4f} ms  (rounds {', '.join('%.4f' % v for v in res[c])})")


if __name__ == "__main__":
    main()
