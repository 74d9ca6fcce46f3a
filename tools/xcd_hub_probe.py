"""Emulate an XCD-sliced hub pass with the shipped SpMM kernel, to price it before building it.

tools/workingset_probe.py: a gather working set that fits one XCD's L2 (4 MiB) runs at
~50 G rows/s, while 16-256 MiB sets (Infinity Cache) run at 14-19 G rows/s, barely above
HBM (12 G rows/s); giving each XCD 1/8 of a 32 MiB set brings it back to 45 G rows/s.
The hub-staged SpMM reads its 64 MiB hub table from every XCD.

Emulation: hub ranks are dealt to 8 slices (rank % 8). For rows of degree >= T, the hub
edges of one (row, slice) pair with >= 2 edges become one "item" (chunked to <= C edges).
Pass 1 runs the items with the shipped kernel, item rows laid out so that workgroup w
(4 items, one per wave) only holds items of slice w % 8, i.e. runs them on XCD w % 8; each
item writes a partial row into P. Pass 2 is the shipped hub kernel over
[remaining edges | refs to the row's partials (value 1.0)], reading the hub table and P
through ONE staged buffer [table | P].

    python tools/xcd_hub_probe.py [--workload cfg2|ns] [--T 64] [--C 128]
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
    ap.add_argument("--T", default="16,64,256")
    ap.add_argument("--C", type=int, default=128)
    ap.add_argument("--slices", type=int, default=8)
    ap.add_argument("--K1", default="0", help="slice only hub ranks < K1 (0: all staged hubs)")
    ap.add_argument("--K", default="0", help="staged hub rows (0: hub_rows_for)")
    ap.add_argument("--M", default="2", help="min hub edges of a (row, slice) item")
    args = ap.parse_args()
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.graph import CsrGraph, from_coo, seg_len_for
    from graphneuralnetwork_amd.ops import hub_rows_for, spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, e = (1_000_000, 10_000_000) if args.workload == "cfg2" else (10_000_000, 100_000_000)
    s, d = rmat_edges(n, e, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n, device=dev)
    del s, d
    F = args.feat
    NS = args.slices
    X = torch.randn(n, F, device=dev)
    bias = torch.randn(F, device=dev)
    Y0 = torch.empty(n, F, device=dev)
    Y = torch.empty(n, F, device=dev)
    lib = _lib.load()
    stream = _lib.stream_handle(dev)
    i64 = torch.int64

    def tm(fn, reps=10):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / reps)
        return statistics.median(ts)

    base = tm(lambda: spmm_forward(g, X, bias, out=Y0))
    print(json.dumps({"workload": args.workload, "nnz": g.nnz, "baseline_ms": round(base, 4)}),
          flush=True)
    sl = seg_len_for(F)

    def hub_call(gr, plan, y, ldy, xh, b, partial):
        pa = plan.args()
        _lib.check(lib.gnn_spmm_csr_hub_f32(
            gr.rowptr.data_ptr(), gr.col.data_ptr(), gr.val.data_ptr(), gr.n_rows, X.data_ptr(),
            F, xh.data_ptr(), F, F, _lib.ptr(b), y.data_ptr(), ldy, plan.seg_len, *pa,
            _lib.ptr(partial), 0, stream), "hub")

    deg = g.rowptr[1:] - g.rowptr[:-1]
    rows_e = torch.repeat_interleave(torch.arange(n, device=dev), deg)
    grid = [(int(kk) or hub_rows_for(n, F), int(t), int(k1), int(mm)) for kk in args.K.split(",")
            for t in args.T.split(",") for k1 in args.K1.split(",") for mm in args.M.split(",")]
    for K, T, K1, M in grid:
        K1 = K1 or K
        hp = g.hub_plan(K)
        c = hp.col_hub.to(i64)
        cand = (c < 0) & (c >= -K1) & (deg[rows_e] >= T)
        eid = torch.nonzero(cand).view(-1)
        k_e = -1 - c[eid]
        s_e = k_e % NS
        key = rows_e[eid] * NS + s_e
        order = torch.argsort(key, stable=True)
        eid, key, s_e = eid[order], key[order], s_e[order]
        ukey, inv, m = torch.unique_consecutive(key, return_inverse=True, return_counts=True)
        moved_g = m >= M
        em = moved_g[inv]
        eid, key, s_e, inv = eid[em], key[em], s_e[em], inv[em]
        # regroup moved edges: group index among moved groups
        gm = torch.cumsum(moved_g.to(i64), 0) - 1
        grp = gm[inv]
        mg = m[moved_g]
        ng = int(mg.numel())
        nch = (mg + args.C - 1) // args.C
        # edge's position within its group
        gstart = torch.cumsum(mg, 0) - mg
        pos_in = torch.arange(eid.numel(), device=dev) - gstart[grp]
        chunk_in = pos_in * nch[grp] // mg[grp]          # balanced chunks
        cstart = torch.cumsum(nch, 0) - nch
        chunk = cstart[grp] + chunk_in                    # chunk id (ordered by row, slice)
        n_chunks = int(nch.sum())
        ch_slice = torch.empty(n_chunks, dtype=i64, device=dev)
        ch_slice[chunk] = s_e
        ch_row = torch.empty(n_chunks, dtype=i64, device=dev)
        ch_row[chunk] = rows_e[eid]
        # index within slice, in chunk order
        j = torch.zeros(n_chunks, dtype=i64, device=dev)
        cnt = torch.bincount(ch_slice, minlength=NS)
        for sidx in range(NS):
            msk = ch_slice == sidx
            j[msk] = torch.arange(int(cnt[sidx]), device=dev)
        per = int(((cnt.max() + 3) // 4) * 4)
        pos = ((j // 4) * NS + ch_slice) * 4 + (j % 4)
        n_pos = per * NS
        # dummies: every unfilled position gets 2 edges to a hub of its slice, value 0
        filled = torch.zeros(n_pos, dtype=torch.bool, device=dev)
        filled[pos] = True
        dpos = torch.nonzero(~filled).view(-1)
        dsl = (dpos // 4) % NS
        p1_rows = torch.cat([pos[chunk], dpos, dpos])
        p1_cols = torch.cat([c[eid], -1 - dsl, -1 - dsl])
        p1_vals = torch.cat([g.val[eid], torch.zeros(2 * dpos.numel(), device=dev)])
        g1 = from_coo(p1_rows, p1_cols, p1_vals, n_pos, K, check=False)
        plan1 = g1.plan(sl)
        assert plan1.n_small == 0 and plan1.n_seg == 0, (plan1.n_small, plan1.n_seg)
        assert torch.equal(plan1.mid_row.to(i64), torch.arange(n_pos, device=dev))
        # pass 2: unmoved edges in order, then refs to the row's chunks
        keep = torch.ones(g.nnz, dtype=torch.bool, device=dev)
        keep[eid] = False
        kid = torch.nonzero(keep).view(-1)
        p2_rows = torch.cat([rows_e[kid], ch_row])
        p2_cols = torch.cat([c[kid], -1 - (K + pos)])
        p2_vals = torch.cat([g.val[kid], torch.ones(n_chunks, device=dev)])
        g2 = from_coo(p2_rows, p2_cols, p2_vals, n, n, check=False)
        plan2 = g2.plan(sl)
        buf = torch.empty(K + n_pos, F, device=dev)
        part1 = torch.empty(max(plan1.n_seg, 1), F, device=dev)
        part2 = torch.empty(max(plan2.n_seg, 1), F, device=dev)
        P = buf[K:]

        def gather():
            _lib.check(lib.gnn_gather_rows_f32(X.data_ptr(), F, n, hp.hub_ids.data_ptr(), K, F,
                                               buf.data_ptr(), F, hp.err.data_ptr(), stream), "g")

        def p1():
            hub_call(g1, plan1, P, F, buf, None, part1)

        def p2():
            hub_call(g2, plan2, Y, F, buf, bias, part2)

        def full():
            gather()
            p1()
            p2()
        t_full = tm(full)
        t_g, t1, t2 = tm(gather), tm(p1), tm(p2)
        full()
        torch.cuda.synchronize()
        err = float((Y - Y0).abs().max() / Y0.abs().max())
        print(json.dumps({"K": K, "T": T, "M": M, "C": args.C, "K1": K1, "moved_edges": int(eid.numel()),
                          "items": n_chunks, "positions": n_pos, "per_slice": cnt.tolist(),
                          "pass2_nnz": g2.nnz, "ms": round(t_full, 4), "gather_ms": round(t_g, 4),
                          "pass1_ms": round(t1, 4), "pass2_ms": round(t2, 4),
                          "speedup": round(base / t_full, 3), "max_rel_err": err}), flush=True)
        del g1, g2, plan1, plan2, buf, part1, part2, P
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
