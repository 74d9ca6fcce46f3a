"""Feature-sliced SpMM probe (tools/fs_probe.hip): does gathering F / SL columns per XCD, so
that an XCD's L2 holds SL x more table rows, beat the library's SpMM at cfg2?

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/fs_probe.hip -o tools/libfs_probe.so  (CPU)
    python tools/fs_probe.py [--nodes 1000000 --edges 10000000] [--sl 1,2,4,8] [--wgs 64,128,256]

Prints per (SL, workgroups per XCD, segment length) the median ms of 20 launches and the max
error against ops.spmm_forward over the same column-ordered graph (timed beside it).
"""
import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def timed(fn, reps, dev):
    s = torch.cuda.current_stream(dev)
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        torch.cuda.synchronize(dev)
        out.append(a.elapsed_time(b))
    return statistics.median(out[2:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=10_000_000)
    ap.add_argument("--sl", default="1,2,4,8")
    ap.add_argument("--wgs", default="128,256")
    ap.add_argument("--seg", default="256")
    ap.add_argument("--short", type=int, default=64)
    ap.add_argument("--reps", type=int, default=22)
    ap.add_argument("--mode", default="items", choices=["items", "split"])
    a = ap.parse_args()
    from graphneuralnetwork_amd.ops import column_order, spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(str(ROOT / "tools" / "libfs_probe.so"))
    lib.fs_probe_run.restype = ctypes.c_int
    lib.fs_probe_run.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 6 + [ctypes.c_int64] + \
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
         ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    s, d = rmat_edges(a.nodes, a.edges, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), a.nodes)
    o = column_order(g, 128)
    ga = g if o is None else o.graph
    F = 128
    X = torch.randn(ga.n_cols, F, device=dev)
    Yref = spmm_forward(ga, X)
    base = timed(lambda: spmm_forward(ga, X, out=Yref), a.reps, dev)
    print(json.dumps({"library_spmm_ms": round(base, 4), "nnz": ga.nnz}), flush=True)
    rp = ga.rowptr
    deg = rp[1:] - rp[:-1]
    short = torch.nonzero(deg <= a.short).flatten().to(torch.int32)
    lrow = torch.nonzero(deg > a.short).flatten()
    stream = torch.cuda.current_stream(dev).cuda_stream
    Y = torch.empty_like(Yref)
    if a.mode == "items":
        lib.fs_probe_items.restype = ctypes.c_int
        lib.fs_probe_items.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int64] + \
            [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
             ctypes.c_void_p]
        n = ga.n_rows
        for L in [int(v) for v in a.seg.split(",")]:
            nseg = torch.where(deg > L, (deg + L - 1) // L, torch.ones_like(deg))
            start = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            start[1:] = torch.cumsum(nseg, 0)
            tot = int(start[-1])
            row = torch.repeat_interleave(torch.arange(n, device=dev), nseg)
            k = torch.arange(tot, device=dev) - start[row]
            b = rp[row] + k * L
            e = torch.minimum(b + L, rp[row + 1])
            islong = deg[row] > L
            lrow = torch.nonzero(deg > L).flatten()
            nls = nseg[lrow]
            lseg = torch.zeros(lrow.numel() + 1, dtype=torch.int64, device=dev)
            lseg[1:] = torch.cumsum(nls, 0)
            # partial index of a long row's segment k: lseg[rank of the row among long rows] + k
            lrank = torch.full((n,), -1, dtype=torch.int64, device=dev)
            lrank[lrow] = torch.arange(lrow.numel(), device=dev)
            pidx = torch.where(islong, lseg[lrank[row].clamp(min=0)] + k, torch.zeros_like(k))
            dst = torch.where(islong, -1 - pidx, row)
            order = torch.argsort(-(e - b), stable=True)
            items = torch.stack([b, e, dst], 1)[order].contiguous()
            part = torch.empty(max(int(lseg[-1]), 1), F, device=dev)
            lrow32 = lrow.to(torch.int32)
            print(json.dumps({"seg": L, "items": tot, "long_rows": lrow.numel(),
                              "partials": int(lseg[-1])}), flush=True)
            for sl in [int(v) for v in a.sl.split(",")]:
                for w in [int(v) for v in a.wgs.split(",")]:
                    def run():
                        rc = lib.fs_probe_items(sl, ga.col.data_ptr(), ga.val.data_ptr(),
                                                X.data_ptr(), Y.data_ptr(), items.data_ptr(), tot,
                                                lrow32.data_ptr(), lseg.data_ptr(), lrow.numel(),
                                                part.data_ptr(), w, ctypes.c_void_p(stream))
                        assert rc == 0, rc
                    Y.fill_(float("nan"))
                    run()
                    torch.cuda.synchronize(dev)
                    err = float((Y - Yref).abs().max())
                    ms = timed(run, a.reps, dev)
                    print(json.dumps({"mode": "items", "sl": sl, "wgs_per_xcd": w, "seg": L,
                                      "ms": round(ms, 4), "vs_library": round(ms / base, 3),
                                      "max_abs_err": err}), flush=True)
        return
    for L in [int(v) for v in a.seg.split(",")]:
        nseg = (deg[lrow] + L - 1) // L
        lseg = torch.zeros(lrow.numel() + 1, dtype=torch.int64, device=dev)
        lseg[1:] = torch.cumsum(nseg, 0)
        n_seg = int(lseg[-1])
        sidx = torch.repeat_interleave(torch.arange(lrow.numel(), device=dev), nseg)
        k = torch.arange(n_seg, device=dev) - lseg[sidx]
        b = rp[lrow[sidx]] + k * L
        e = torch.minimum(b + L, rp[lrow[sidx] + 1])
        seg = torch.stack([b, e], 1).contiguous()
        part = torch.empty(n_seg, F, device=dev)
        lrow32 = lrow.to(torch.int32)
        for sl in [int(v) for v in a.sl.split(",")]:
            for w in [int(v) for v in a.wgs.split(",")]:
                def run():
                    rc = lib.fs_probe_run(sl, rp.data_ptr(), ga.col.data_ptr(), ga.val.data_ptr(),
                                          X.data_ptr(), Y.data_ptr(), short.data_ptr(), short.numel(),
                                          seg.data_ptr(), n_seg, lrow32.data_ptr(), lseg.data_ptr(),
                                          lrow.numel(), part.data_ptr(), w, ctypes.c_void_p(stream))
                    assert rc == 0, rc
                Y.fill_(float("nan"))
                run()
                torch.cuda.synchronize(dev)
                err = float((Y - Yref).abs().max())
                ms = timed(run, a.reps, dev)
                print(json.dumps({"sl": sl, "wgs_per_xcd": w, "seg": L, "ms": round(ms, 4),
                                  "vs_library": round(ms / base, 3), "max_abs_err": err}), flush=True)


if __name__ == "__main__":
    main()
