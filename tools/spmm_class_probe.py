"""Where the SpMM time goes, by row class: the cfg2 / north-star graph with only the rows
of one degree class kept (every other row emptied, so it costs one packed small-row store),
timed with the default kernel and hub staging.

    python tools/spmm_class_probe.py [--workload cfg2|ns] [--feat 128]
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
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--classes", default="0-1,2-4,5-16,17-64,65-384,385-1000000000")
    args = ap.parse_args()
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, e = (1_000_000, 10_000_000) if args.workload == "cfg2" else (10_000_000, 100_000_000)
    s, d = rmat_edges(n, e, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n, device=dev)
    del s, d
    F = args.feat
    X = torch.randn(n, F, device=dev)
    Y = torch.empty(n, F, device=dev)
    deg = g.rowptr[1:] - g.rowptr[:-1]

    def timed(gr, reps=10):
        for _ in range(3):
            spmm_forward(gr, X, out=Y)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                spmm_forward(gr, X, out=Y)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / reps)
        return statistics.median(ts)

    full = timed(g)
    print(json.dumps({"workload": args.workload, "class": "all", "rows": n, "nnz": g.nnz,
                      "ms": full}), flush=True)
    rows_of_edge = torch.repeat_interleave(torch.arange(n, device=dev), deg)
    for c in args.classes.split(","):
        lo, hi = (int(v) for v in c.split("-"))
        keep_row = (deg >= lo) & (deg <= hi)
        keep = keep_row[rows_of_edge]
        kd = torch.where(keep_row, deg, torch.zeros_like(deg))
        rp = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(kd, 0, out=rp[1:])
        sub = CsrGraph(rp, g.col[keep].contiguous(), g.val[keep].contiguous(), n, n)
        ms = timed(sub)
        print(json.dumps({"workload": args.workload, "class": c, "rows": int(keep_row.sum()),
                          "nnz": sub.nnz, "ms": ms, "edges_per_ns": sub.nnz / ms / 1e6}),
              flush=True)
        del sub, keep, kd, rp


if __name__ == "__main__":
    main()
