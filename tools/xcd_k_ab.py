"""A/B in one process of the XCD-sliced SpMM's hub-row count K over the column-degree-ordered
graph (the shipped path: ops.column_order, hub rows read in place): K = XCD_HUB_ROWS with
XCD_HUB_BYTES lifted, output checked against the default K's.

    python tools/xcd_k_ab.py --workload cfg2|ns [--ks 262144,393216,524288]     (GPU)
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timed(fn, reps=10, rounds=7):
    out = []
    for _ in range(rounds):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) / reps)
    return round(statistics.median(out), 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--ks", default="262144,393216,524288,786432")
    ap.add_argument("--param", default="XCD_HUB_ROWS",
                    help="the ops knob swept with --ks (e.g. XCD_MIN_DEG, XCD_CHUNK)")
    a = ap.parse_args()
    import bench
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.ops import column_order, spmm_forward
    dev = torch.device("cuda:0")
    wl = bench.WORKLOADS[a.workload]
    F = wl.get("feat", 128)
    g = bench.build_graph(wl["nodes"], wl["edges"], dev, 0, 1)
    ga = column_order(g, F).graph
    X = torch.randn(g.n_cols, F, device=dev)
    Y = torch.empty(g.n_rows, F, device=dev)
    b = torch.randn(F, device=dev)
    if a.param == "XCD_HUB_ROWS":
        ops.XCD_HUB_BYTES = 1 << 40
    res, ref = {"workload": a.workload, "param": a.param}, None
    for rnd in range(2):  # two interleaved rounds
        for k in [int(v) for v in a.ks.split(",")]:
            setattr(ops, a.param, k)
            fn = lambda: spmm_forward(ga, X, b, out=Y)  # noqa: E731
            fn()
            if ref is None:
                ref = Y.clone()
            err = float(((Y - ref).abs().max() / ref.abs().max()))
            t = timed(fn)
            res.setdefault(str(k), []).append(t)
            res[f"{k}_err"] = err
            print(json.dumps({"k": k, "ms": t, "rel_err_vs_first": err}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
