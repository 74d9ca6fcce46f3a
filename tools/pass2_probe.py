"""Where the XCD-sliced SpMM step spends its time (cfg2 / north star): each launch timed alone,
and each pass again with every column folded into a 1 MiB set (L2-resident gathers, same row
structure, same instruction stream) -- the gap between the two is what the memory side costs;
what is left is the kernel's own latency / issue cost.

    python tools/pass2_probe.py [--workload cfg2|ns] [--fold 2048]
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


def fold(g, m):
    """The same CSR with column c -> c % m and staged id -1-r -> -1-(r % m)."""
    from graphneuralnetwork_amd.graph import CsrGraph
    c = g.col.to(torch.int64)
    neg = c < 0
    f = torch.where(neg, -1 - ((-1 - c) % m), c % m).to(torch.int32)
    return CsrGraph(g.rowptr, f.contiguous(), g.val, g.n_rows, g.n_cols)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--fold", type=int, default=2048)
    ap.add_argument("--feat", type=int, default=128)
    a = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import seg_len_for, staged_plan
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n, e = (1_000_000, 10_000_000) if a.workload == "cfg2" else (10_000_000, 100_000_000)
    dev = torch.device("cuda:0")
    s, d = rmat_edges(n, e, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    F = a.feat
    X = torch.randn(n, F, device=dev)
    Y = torch.empty(n, F, device=dev)
    full = timed(lambda: ops.spmm_forward(g, X, None, out=Y))
    lib = _lib.load()
    seg = seg_len_for(F)
    kx = ops.xcd_hub_rows_for(g.n_cols, F)
    xp = g.xcd_hub_plan(kx, ops.XCD_MIN_DEG, min(ops.XCD_CHUNK, seg))
    k = xp.k
    buf = torch.empty((k + xp.n_pos, F), device=dev)
    stream = _lib.stream_handle(dev)
    hp = xp.hub

    def hub_copy():
        _lib.check(lib.gnn_gather_rows_f32(X.data_ptr(), F, n, hp.hub_ids.data_ptr(), k, F,
                                           buf.data_ptr(), F, hp.err.data_ptr(), stream), "copy")

    p1 = xp.items.plan(seg)
    p2 = xp.rest_plan(seg)
    part = torch.empty((max(p2.n_seg, 1), F), device=dev)

    def pass1(items=xp.items, plan=p1):
        ops._spmm_hub_call(lib, items, items.col, plan, plan.args(), X, buf, F, None, buf[k:], F,
                           None, 0, stream, "p1")

    def pass2(rest=xp.rest, plan=p2):
        ops._spmm_hub_call(lib, rest, rest.col, plan, plan.args(), X, buf, F, None, Y, F,
                           part if plan.n_seg else None, 0, stream, "p2")

    res = {"step": full, "hub_copy": timed(hub_copy), "pass1": timed(pass1), "pass2": timed(pass2)}
    items_f = fold(xp.items, a.fold)
    rest_f = fold(xp.rest, a.fold)
    p2f = staged_plan(rest_f, seg)
    res["pass1_folded"] = timed(lambda: pass1(items_f, p1))
    res["pass2_folded"] = timed(lambda: pass2(rest_f, p2f))
    deg = (xp.rest.rowptr[1:] - xp.rest.rowptr[:-1])
    print(f"workload {a.workload} F={F} k={k} items {xp.n_items} (positions {xp.n_pos}) "
          f"rest nnz {xp.rest.nnz} rows {xp.rest.n_rows}: mid {p2.n_mid} small {p2.n_small} "
          f"seg {p2.n_seg}; rest degree mean {float(deg.float().mean()):.2f}")
    for kk, v in res.items():
        print(f"  {kk:14s} {v:8.4f} ms")


if __name__ == "__main__":
    main()
