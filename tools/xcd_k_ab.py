"""Interleaved A/B of the XCD hub count K (ops.XCD_HUB_ROWS) on the column-ordered graph, the
default path of bench.py (hub rows read in place; one plan per K, cached on the graph).

    python tools/xcd_k_ab.py [--workload cfg2|ns] [--ks 196608,262144,327680] [--rounds 6]
    python tools/xcd_k_ab.py --min-degs 64,96,128,192      (ops.XCD_MIN_DEG at the default K)
    python tools/xcd_k_ab.py --knob TASK_COST --values 128,256,512   (any integer ops knob)
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
    ap.add_argument("--ks", default="196608,262144,327680,393216")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--min-degs", default="", help="sweep ops.XCD_MIN_DEG instead of K")
    ap.add_argument("--phases", default="", help="sweep ops.XCD_PHASES instead of K")
    ap.add_argument("--knob", default="", help="sweep this integer ops knob over --values")
    ap.add_argument("--values", default="")
    a = ap.parse_args()
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, e = (1_000_000, 10_000_000) if a.workload == "cfg2" else (10_000_000, 100_000_000)
    s, d = rmat_edges(n, e, 0)
    g = ops.column_order(gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n),
                         128).graph
    X = torch.randn(n, 128, device=dev)
    Y = torch.empty(n, 128, device=dev)
    ref = ops.spmm_forward(g, X).clone()
    if a.knob:
        a.min_degs = a.phases = ""
    sweep_deg, sweep_ph = bool(a.min_degs), bool(a.phases)
    src = a.values if a.knob else a.min_degs if sweep_deg else a.phases if sweep_ph else a.ks
    ks = [int(v) for v in src.split(",")]
    times = {k: [] for k in ks}
    for r in range(a.rounds):
        for k in ks:
            if a.knob:
                setattr(ops, a.knob, k)
            elif sweep_deg:
                ops.XCD_MIN_DEG = k
            elif sweep_ph:
                ops.XCD_PHASES = k
            else:
                ops.XCD_HUB_ROWS, ops.XCD_HUB_BYTES = k, k * 512
            ops.spmm_forward(g, X, out=Y)
            torch.cuda.synchronize()
            if r == 0:
                err = float(((Y - ref).abs() / (ref.abs() + 1e-3)).max())
                print(json.dumps({"k": k, "max_rel_err_vs_default": err}), flush=True)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(5):
                ops.spmm_forward(g, X, out=Y)
            ev[1].record()
            torch.cuda.synchronize()
            times[k].append(ev[0].elapsed_time(ev[1]) / 5)
    print(json.dumps({"workload": a.workload, "swept": a.knob or ("XCD_MIN_DEG" if sweep_deg else "XCD_PHASES" if sweep_ph else "K"),
                      "median_ms": {k: round(statistics.median(t), 4) for k, t in times.items()}}))


if __name__ == "__main__":
    main()
