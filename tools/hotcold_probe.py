"""Probe: does splitting the SpMM by column hotness let the hot feature rows live in the
Infinity Cache?  Interleaved A/B in one process.

    python tools/hotcold_probe.py [--workload cfg2|ns] [--feat 128] [--ks 65536,262144]

Variants (Y = A X + b, same output):
  base     one launch over the whole CSR
  hot1     pass 1 = edges into the K highest-degree columns (writes Y + b),
           pass 2 = the remaining edges (accumulates into Y)
  cold1    the same two passes, cold first
  hotc     hot1 with the hot rows of X first compacted into a [K, F] buffer (the
           index_select is inside the timed step)
Each pass is also timed alone.
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def split_by_columns(g, hot_mask):
    from graphneuralnetwork_amd.graph import CsrGraph
    n = g.n_rows
    deg = g.rowptr[1:] - g.rowptr[:-1]
    rows = torch.repeat_interleave(torch.arange(n, device=g.rowptr.device), deg)
    m = hot_mask[g.col.long()]
    out = []
    for sel in (m, ~m):
        cnt = torch.bincount(rows[sel], minlength=n)
        rp = torch.zeros(n + 1, dtype=torch.int64, device=g.rowptr.device)
        rp[1:] = torch.cumsum(cnt, 0)
        out.append(CsrGraph(rp, g.col[sel].contiguous(), g.val[sel].contiguous(), n, g.n_cols))
    del rows, m
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ns")
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--ks", default="65536,131072,262144,524288")
    ap.add_argument("--rounds", type=int, default=6)
    args = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.graph import CsrGraph
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
    ref = spmm_forward(g, X, b).clone()
    nbytes = g.nnz * (8 + 4 * F) + n * (8 + 4 * F)
    stream = torch.cuda.current_stream(dev)
    col_deg = torch.bincount(g.col.long(), minlength=n)
    order = torch.argsort(col_deg, descending=True)
    csum = torch.cumsum(col_deg[order], 0)

    variants = {"base": lambda: spmm_forward(g, X, b, out=Y)}
    for K in map(int, args.ks.split(",")):
        hot_ids = order[:K].sort().values
        mask = torch.zeros(n, dtype=torch.bool, device=dev)
        mask[hot_ids] = True
        gh, gc = split_by_columns(g, mask)
        rank = torch.full((n,), -1, dtype=torch.int32, device=dev)
        rank[hot_ids] = torch.arange(K, dtype=torch.int32, device=dev)
        ghc = CsrGraph(gh.rowptr, rank[gh.col.long()].contiguous(), gh.val, n, K)
        hot_ids32 = hot_ids
        Xh = torch.empty(K, F, device=dev)
        cover = float(csum[K - 1]) / g.nnz
        print(json.dumps({"K": K, "hot_nnz": gh.nnz, "cold_nnz": gc.nnz, "cover": cover,
                          "hot_MiB": K * 4 * F / 2**20}), flush=True)

        def hot1(gh=gh, gc=gc):
            spmm_forward(gh, X, b, out=Y)
            spmm_forward(gc, X, None, out=Y, accumulate=True)

        def cold1(gh=gh, gc=gc):
            spmm_forward(gc, X, b, out=Y)
            spmm_forward(gh, X, None, out=Y, accumulate=True)

        def hotc(ghc=ghc, gc=gc, ids=hot_ids32, Xh=Xh):
            torch.index_select(X, 0, ids, out=Xh)
            spmm_forward(ghc, Xh, b, out=Y)
            spmm_forward(gc, X, None, out=Y, accumulate=True)

        variants[f"hot1_K{K}"] = hot1
        variants[f"cold1_K{K}"] = cold1
        variants[f"hotc_K{K}"] = hotc
        variants[f"passhot_K{K}"] = (lambda gh=gh: spmm_forward(gh, X, b, out=Y))
        variants[f"passcold_K{K}"] = (lambda gc=gc: spmm_forward(gc, X, None, out=Y,
                                                                 accumulate=True))
    torch.cuda.empty_cache()
    for name, fn in variants.items():  # correctness + warm-up (plans are built here)
        fn()
        torch.cuda.synchronize()
        if not name.startswith("pass"):
            err = float((Y - ref).abs().max() / ref.abs().max())
            assert err < 1e-5, (name, err)
    times = {k: [] for k in variants}
    for _ in range(args.rounds):
        for name, fn in variants.items():
            a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fn()
            a.record(stream)
            for _ in range(3):
                fn()
            c.record(stream)
            torch.cuda.synchronize()
            times[name].append(a.elapsed_time(c) / 3)
    for name, t in times.items():
        med = statistics.median(t)
        print(json.dumps({"variant": name, "median_ms": med, "min_ms": min(t),
                          "algo_GBps": nbytes / (med / 1e3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
