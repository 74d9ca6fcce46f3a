"""Price the dense-corner split of the SpMM: in the degree order the top
T x T ids of the R-MAT matrix are dense (cfg2: 24 % at T = 2048); their edges could run as one
dense GEMM instead of T-row gathers. Times, interleaved in one process: the SpMM over A P^T as
benchmarked, the SpMM over A P^T minus the corner edges (its own plans), and the fp32 dense
GEMM of the corner block (torch.mm, hipBLASLt). No product code.

    python tools/corner_probe.py [--workload cfg2|ns] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2", choices=("cfg2", "ns"))
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import bench
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import column_order, spmm_forward
    dev = torch.device("cuda:0")
    wl = bench.WORKLOADS[a.workload]
    F = 128
    g = bench.build_graph(wl["nodes"], wl["edges"], dev, 0, 1)
    order = column_order(g, F)
    ga = order.graph
    n = g.n_rows
    X = torch.randn(n, F, device=dev)
    Y = torch.empty(n, F, device=dev)
    spmm_forward(ga, X, None, out=Y)
    base = timed(lambda: spmm_forward(ga, X, None, out=Y), a.reps)
    rows = torch.repeat_interleave(torch.arange(n, device=dev), ga.rowptr[1:] - ga.rowptr[:-1])
    rrank = order.inv[rows]  # the row's degree rank (symmetric graph: same order)
    res = {"workload": a.workload, "as_built_ms": base}
    for T in (1024, 2048, 4096, 8192):
        corner = (rrank < T) & (ga.col < T)
        keep = ~corner
        kr = rows[keep]
        rowptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        rowptr[1:] = torch.cumsum(torch.bincount(kr, minlength=n), 0)
        rest = CsrGraph(rowptr, ga.col[keep].contiguous(), ga.val[keep].contiguous(), n, n)
        spmm_forward(rest, X, None, out=Y)
        t_rest = timed(lambda: spmm_forward(rest, X, None, out=Y), a.reps)
        D = torch.zeros(T, T, device=dev)
        D[rrank[corner], ga.col[corner].to(torch.int64)] = ga.val[corner]
        Xt = X[:T].contiguous()
        t_gemm = timed(lambda: torch.mm(D, Xt), a.reps)
        res[f"T{T}"] = {"corner_edges": int(corner.sum()), "rest_ms": t_rest, "gemm_ms": t_gemm,
                        "sum_ms": t_rest + t_gemm, "gain": 1 - (t_rest + t_gemm) / base}
        print(json.dumps(res[f"T{T}"]), flush=True)
        del rest, D, corner, keep, kr
        torch.cuda.empty_cache()
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
