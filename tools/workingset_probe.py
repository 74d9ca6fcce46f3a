"""Gather rate vs working-set size and XCD locality (what an L2-aware hub layout could buy).

Synthetic CSR: R rows of exactly D edges (all "mid" rows: one wave per row, 4 waves per
workgroup, so row r runs in workgroup r // 4 and -- with the round-robin dispatch of
workgroups over the 8 XCDs -- on XCD (r // 4) % 8). X is the 10M x F table of the north
star. Column patterns over a working set of S rows:

  scattered  S rows picked at random over the whole 10M-row table
  compact    rows 0..S-1
  xcd        rows 0..S-1, but a row on XCD x only gathers from slice x (S/8 rows): each
             XCD's L2 sees 1/8 of the set

Reported: ms per SpMM, G gathered rows/s, algorithmic GB/s.

    python tools/workingset_probe.py [--feat 128] [--deg 64] [--nnz 20000000]
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
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--deg", type=int, default=64)
    ap.add_argument("--nnz", type=int, default=20_000_000)
    ap.add_argument("--table", type=int, default=10_000_000)
    ap.add_argument("--sizes", default="4096,8192,32768,65536,131072,524288,2097152,10000000")
    ap.add_argument("--op", default="spmm", choices=["spmm", "gat"],
                    help="gat: the GAT aggregation (dense softmax + ELU, 8 heads x feat/8; "
                         "gathers a Wh row and an er entry per edge)")
    args = ap.parse_args()
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import gat_aggregate, spmm_forward
    dev = torch.device("cuda:0")
    F, D = args.feat, args.deg
    R = args.nnz // D
    nnz = R * D
    X = torch.randn(args.table, F, device=dev)
    Y = torch.empty(R, F, device=dev)
    rowptr = torch.arange(0, nnz + 1, D, device=dev, dtype=torch.int64)
    val = torch.full((nnz,), 1.0 / D, device=dev)
    xcd_of_row = (torch.arange(R, device=dev) // 4) % 8
    xcd_of_edge = xcd_of_row.repeat_interleave(D)
    gen = torch.Generator(device=dev).manual_seed(0)

    if args.op == "gat":
        H = 8
        el = torch.randn(R, H, device=dev)
        er = torch.randn(args.table, H, device=dev)

        def run(g):
            gat_aggregate(g, X, el, er, H, F // H, 0.2, 0, "elu", out=Y, hubs=0)
    else:
        def run(g):
            spmm_forward(g, X, out=Y, hubs=0)

    def timed(g, reps=10):
        for _ in range(3):
            run(g)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                run(g)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / reps)
        return statistics.median(ts)

    res = []
    alg = nnz * (8 + 4 * F) + R * (8 + 4 * F)
    for S in (int(s) for s in args.sizes.split(",")):
        S = min(S, args.table)
        r = torch.randint(0, S, (nnz,), device=dev, generator=gen)
        pats = {}
        pick = torch.randperm(args.table, device=dev, generator=gen)[:S]
        pats["scattered"] = pick[r]
        pats["compact"] = r
        if S >= 8 and S < args.table:
            sl = S // 8
            pats["xcd"] = xcd_of_edge * sl + torch.randint(0, sl, (nnz,), device=dev, generator=gen)
        for name, col in pats.items():
            g = CsrGraph(rowptr, col.to(torch.int32), val, R, args.table)
            ms = timed(g)
            line = {"S": S, "set_MiB": S * 4 * F / 2**20, "pattern": name, "ms": round(ms, 4),
                    "G_rows_per_s": round(nnz / ms / 1e6, 2), "alg_GBps": round(alg / ms / 1e6)}
            res.append(line)
            print(json.dumps(line), flush=True)
            del g
        del r, pats, pick
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
