"""Pass overlap probe for the XCD-sliced SpMM (ops._spmm_xcd_direct) at cfg2 / the north star.

Pass 1 (hub items -> partial rows) and pass 2 (the rest + partial refs) run one after the
other today. Only the rows of pass 2 that hold a partial ref need pass 1's output; the others
could run on a second stream while pass 1 runs. This splits the rest graph into A (rows without
a partial ref) and B (rows with one), both launched with EPI_SKIP_EMPTY so each writes only its
own rows, and times

  seq      the library's spmm_forward (pass 1, pass 2)
  overlap  pass 1 on stream 1 || pass 2A on stream 2, then pass 2B after pass 1
  split    pass 1, pass 2A, pass 2B on one stream (the cost of splitting alone)

and checks the output against spmm_forward.

    python tools/overlap_probe.py [--workload cfg2|ns] [--reps 20]
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
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from graphneuralnetwork_amd import _lib, ops
    from graphneuralnetwork_amd.graph import CsrGraph, seg_len_for
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, m = (1_000_000, 10_000_000) if a.workload == "cfg2" else (10_000_000, 100_000_000)
    F = 128
    s, d = rmat_edges(n, m, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    ga = ops.column_order(g, F).graph
    X = torch.randn(ga.n_cols, F, device=dev)
    Yref = ops.spmm_forward(ga, X)
    seg = seg_len_for(F)
    chunk = min(ops.XCD_CHUNK, seg)
    kx = ops.xcd_hub_rows_for(ga.n_cols, F)
    xp = ga.xcd_hub_plan(kx, ops.XCD_MIN_DEG, chunk, ops.XCD_PHASES, ops.XCD_ITEM_ROWS,
                         ops.XCD_SMALL_ITEM)
    items, rest = xp.direct()
    deg = rest.rowptr[1:] - rest.rowptr[:-1]
    row_of = torch.repeat_interleave(torch.arange(rest.n_rows, device=dev), deg)
    has_ref = torch.zeros(rest.n_rows, dtype=torch.bool, device=dev)
    has_ref[row_of[rest.col < 0]] = True

    def sub(keep_row):
        keep = keep_row[row_of]
        rp = torch.zeros(rest.n_rows + 1, dtype=torch.int64, device=dev)
        rp[1:] = torch.cumsum(torch.where(keep_row, deg, torch.zeros_like(deg)), 0)
        return CsrGraph(rp, rest.col[keep].contiguous(), rest.val[keep].contiguous(), rest.n_rows,
                        rest.n_cols)
    A, B = sub(~has_ref), sub(has_ref)
    print(json.dumps({"workload": a.workload, "items": items.n_rows, "rest_nnz": rest.nnz,
                      "A_rows": int((~has_ref).sum()), "A_nnz": A.nnz,
                      "B_rows": int(has_ref.sum()), "B_nnz": B.nnz}), flush=True)
    lib = _lib.load()
    part = torch.empty((xp.n_pos, F), device=dev)
    p1 = items.plan(seg)
    tA = A.task_plan(seg, ops.TASK_MAX_DEG, ops.TASK_COST)
    tB = B.task_plan(seg, ops.TASK_MAX_DEG, ops.TASK_COST)
    partA = torch.empty((max(tA.base.n_seg, 1), F), device=dev)
    partB = torch.empty((max(tB.base.n_seg, 1), F), device=dev)
    Y = torch.empty_like(Yref)
    flags = _lib.EPI_SKIP_EMPTY
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    cur = torch.cuda.current_stream(dev)

    def pass1(st):
        _lib.check(lib.gnn_spmm_csr_f32(
            items.rowptr.data_ptr(), items.col.data_ptr(), items.val.data_ptr(), items.n_rows,
            X.data_ptr(), X.stride(0), F, None, part.data_ptr(), F, p1.seg_len, *p1.args(),
            None, 0, st), "pass 1")

    def pass2(gr, tp, pt, st):
        ops._spmm_tasks_call(lib, gr, gr.col, tp, X, part, F, None, Y, F,
                             pt if tp.base.n_seg else None, flags, st, "pass 2")

    def split():
        h = cur.cuda_stream
        pass1(h)
        pass2(A, tA, partA, h)
        pass2(B, tB, partB, h)

    def overlap():
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        pass1(s1.cuda_stream)
        pass2(A, tA, partA, s2.cuda_stream)
        s2.wait_stream(s1)
        pass2(B, tB, partB, s2.cuda_stream)
        cur.wait_stream(s2)

    def seq():
        ops.spmm_forward(ga, X, out=Y)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
            fn()
            e1.record(cur)
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts)

    res = {}
    for rnd in range(3):
        for name, fn in (("seq", seq), ("split", split), ("overlap", overlap)):
            Y.fill_(float("nan"))
            fn()
            torch.cuda.synchronize(dev)
            err = float((Y - Yref).abs().max())
            res.setdefault(name, []).append(timed(fn))
            if rnd == 0:
                print(json.dumps({name: "check", "max_abs_err": err,
                                  "bit_equal": bool(torch.equal(Y, Yref))}), flush=True)
    print(json.dumps({k: round(statistics.median(v), 4) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
