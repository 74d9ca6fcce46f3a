"""Interleaved A/B of the SpMM hub-staging size (ops.spmm_forward(hubs=K)) at one shape.

    python tools/hub_ab.py [--workload cfg2|ns] [--feat 128] [--ks 0,16384,65536,...] [--op spmm|gat]

--op gat: the GAT aggregation (ops.gat_aggregate, dense softmax + ELU, 8 heads x feat/8)
with staged Wh and er rows.

K = 0 is the unstaged kernel; every K must give bit-identical output (same edge order,
the gathered values are copies). Times include the per-call hub-row copy.
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
    ap.add_argument("--workload", default="ns")
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--ks", default="0,16384,32768,65536,131072,262144,1048576")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--op", default="spmm", choices=["spmm", "gat"])
    args = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import gat_aggregate, spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    _lib.load()
    dev = torch.device("cuda:0")
    n, e = (1_000_000, 10_000_000) if args.workload == "cfg2" else (10_000_000, 100_000_000)
    s, d = rmat_edges(n, e, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n, device=dev)
    del s, d
    F = args.feat
    X = torch.randn(n, F, device=dev)
    b = torch.randn(F, device=dev)
    Y = torch.empty(n, F, device=dev)
    nbytes = g.nnz * (8 + 4 * F) + n * (8 + 4 * F)
    if args.op == "gat":
        H = 8
        el, er = torch.randn(n, H, device=dev), torch.randn(n, H, device=dev)
        nbytes = g.nnz * (4 + 4 * H + 4 * F) + n * (8 + 4 * H + 4 * F)

        def spmm_forward(g, X, b, out, hubs):  # noqa: F811 -- same harness, GAT op
            return gat_aggregate(g, X, el, er, H, F // H, 0.2, 0, activation="elu", out=out,
                                 hubs=hubs)
    ref = spmm_forward(g, X, b, out=torch.empty_like(Y), hubs=0).clone()
    stream = torch.cuda.current_stream(dev)
    ks = [int(k) for k in args.ks.split(",")]
    for k in ks:
        spmm_forward(g, X, b, out=Y, hubs=k)
        torch.cuda.synchronize()
        assert torch.equal(Y, ref), f"hubs={k}: output differs from the unstaged kernel"
    print(json.dumps({"op": args.op, "workload": args.workload, "feat": F, "nnz": g.nnz, "bitexact": True}),
          flush=True)
    times = {k: [] for k in ks}
    for _ in range(args.rounds):
        for k in ks:
            a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            spmm_forward(g, X, b, out=Y, hubs=k)
            a.record(stream)
            for _ in range(3):
                spmm_forward(g, X, b, out=Y, hubs=k)
            c.record(stream)
            torch.cuda.synchronize()
            times[k].append(a.elapsed_time(c) / 3)
    for k, t in times.items():
        med = statistics.median(t)
        print(json.dumps({"hubs": k, "hub_MiB": k * 4 * F / 2**20, "median_ms": med,
                          "min_ms": min(t), "algo_GBps": nbytes / (med / 1e3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
