"""Interleaved A/B: one full-width SpMM vs the same SpMM done in feature-column passes.

    python tools/fchunk_ab.py [--workload cfg2|ns] [--feat 128] [--variants 128:-1,32:0,...]

A variant W:K runs F/W passes, pass c computing Y[:, c:c+W] = A X[:, c:c+W] (+ b[c:c+W])
with K staged hub rows (-1 = the default rule, 0 = none). The idea under test: a pass
gathers W*4-byte row slices, so the per-XCD L2 (4 MiB) holds 512/W/4 times more of the hot
rows than at full width, at the price of re-reading the CSR once per pass.
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
    ap.add_argument("--variants", default="128:-1,64:0,64:131072,32:0,32:131072,32:32768,16:0")
    ap.add_argument("--rounds", type=int, default=6)
    args = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import spmm_forward
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
    variants = [tuple(int(v) for v in t.split(":")) for t in args.variants.split(",")]

    def run(w, k):
        hubs = None if k < 0 else k
        for c in range(0, F, w):
            spmm_forward(g, X[:, c:c + w], b[c:c + w], out=Y[:, c:c + w], hubs=hubs)

    ref = spmm_forward(g, X, b, hubs=0).clone()
    for w, k in variants:
        Y.zero_()
        run(w, k)
        torch.cuda.synchronize()
        err = float((Y - ref).abs().max() / ref.abs().max())
        print(json.dumps({"variant": f"{w}:{k}", "max_rel_err": err}), flush=True)
        assert err < 1e-5
    stream = torch.cuda.current_stream(dev)
    times = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            run(*v)
            a.record(stream)
            for _ in range(3):
                run(*v)
            c.record(stream)
            torch.cuda.synchronize()
            times[v].append(a.elapsed_time(c) / 3)
    for (w, k), t in times.items():
        med = statistics.median(t)
        print(json.dumps({"workload": args.workload, "width": w, "passes": F // w, "hubs": k,
                          "median_ms": med, "min_ms": min(t),
                          "algo_GBps": nbytes / (med / 1e3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
