"""Interleaved A/B of the XCD-sliced hub staging (ops.spmm_forward xcd=True) against the
single-pass hub staging, at one shape, over (hub rows K, min row degree, item chunk).

    python tools/xcd_ab.py [--workload cfg2|ns] [--feat 128] [--ks 131072,262144]
                           [--degs 64,128,256] [--chunks 128] [--phases 1,2,4]

Every variant is checked against the unstaged kernel (fp32 rounding) before timing. Times
include the per-call hub-row copy and both passes.
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
    ap.add_argument("--ks", default="131072,262144")
    ap.add_argument("--degs", default="64,128,256")
    ap.add_argument("--chunks", default="128")
    ap.add_argument("--phases", default="1",
                    help="slices per XCD run one after another (ops.XCD_PHASES)")
    ap.add_argument("--item-rows", default="0",
                    help="items read only the hottest N hub rows (ops.XCD_ITEM_ROWS; 0 = all)")
    ap.add_argument("--small-items", default="0",
                    help="rows below the degree threshold get items for slices with >= N hub "
                         "edges (ops.XCD_SMALL_ITEM; 0 = off)")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--op", default="spmm", choices=["spmm", "gat"],
                    help="gat: the cfg3 GAT aggregation (dense softmax + ELU, 8 heads x F/8)")
    args = ap.parse_args()
    from graphneuralnetwork_amd import _lib, ops
    from graphneuralnetwork_amd.ops import gat_aggregate, hub_rows_for, spmm_forward
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
    k0 = hub_rows_for(n, F)
    if args.op == "gat":
        H = 8
        el, er = torch.randn(n, H, device=dev), torch.randn(n, H, device=dev)
        nbytes = g.nnz * (4 + 4 * H + 4 * F) + n * (8 + 4 * H + 4 * F)
        k0 = hub_rows_for(n, F + H)

        def spmm_forward(g, X, b, out=None, hubs=None, xcd=None):  # noqa: F811 -- GAT op
            return gat_aggregate(g, X, el, er, H, F // H, 0.2, 0, activation="elu", out=out,
                                 hubs=hubs, xcd=xcd)
    ref = spmm_forward(g, X, b, hubs=0)
    variants = {f"single K={k0}": dict(hubs=k0, xcd=False)}
    for k in (int(v) for v in args.ks.split(",")):
        for dg in (int(v) for v in args.degs.split(",")):
            for ch in (int(v) for v in args.chunks.split(",")):
                for ph in (int(v) for v in args.phases.split(",")):
                    for ik in (int(v) or None for v in args.item_rows.split(",")):
                        for si in (int(v) or None for v in args.small_items.split(",")):
                            variants[f"xcd K={k} deg>={dg} chunk={ch} phases={ph} items<{ik} "
                                     f"small>={si}"] = dict(hubs=k, xcd=True, deg=dg, chunk=ch,
                                                            phases=ph, ik=ik, si=si)

    def call(v):
        if v.get("xcd"):
            ops.XCD_MIN_DEG, ops.XCD_CHUNK = v["deg"], v["chunk"]
            ops.XCD_PHASES, ops.XCD_ITEM_ROWS = v["phases"], v["ik"]
            ops.XCD_SMALL_ITEM = v["si"]
        return spmm_forward(g, X, b, out=Y, hubs=v["hubs"], xcd=v["xcd"])

    scale = float(ref.abs().max())
    for name, v in variants.items():
        call(v)
        torch.cuda.synchronize()
        err = float((Y - ref).abs().max()) / scale
        assert err < 1e-5, (name, err)
        v["err"] = err
        if v.get("xcd") and args.op == "spmm":
            xp = g.xcd_hub_plan(min(v["hubs"], n), v["deg"], min(v["chunk"], ops.seg_len_for(F)),
                                v["phases"], v["ik"], v["si"])
            v["items"] = xp.n_items if xp is not None else 0
    print(json.dumps({"op": args.op, "workload": args.workload, "feat": F, "nnz": g.nnz}),
          flush=True)
    stream = torch.cuda.current_stream(dev)
    times = {k: [] for k in variants}
    for _ in range(args.rounds):
        for name, v in variants.items():
            a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            call(v)
            a.record(stream)
            for _ in range(3):
                call(v)
            c.record(stream)
            torch.cuda.synchronize()
            times[name].append(a.elapsed_time(c) / 3)
    for name, t in times.items():
        med = statistics.median(t)
        print(json.dumps({"variant": name, "median_ms": round(med, 4), "min_ms": round(min(t), 4),
                          "algo_GBps": round(nbytes / (med / 1e3) / 1e9),
                          "max_rel_err": variants[name]["err"],
                          "items": variants[name].get("items")}), flush=True)


if __name__ == "__main__":
    main()
