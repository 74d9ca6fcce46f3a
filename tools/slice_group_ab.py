"""A/B of the XCD hub-slice assignment granularity (plan_build.hip GNN_XCD_SLICE_GROUP): hub
rank r goes to slice (r / G) % 8. G = 1 deals consecutive ranks round-robin, so one XCD's hub
rows sit 8 rows (4 KiB at F = 128) apart in X; larger G keeps G rows of a slice together.
Measured (profiles/r04sg_slice_group_ab.log): cfg2 G = 1 0.8956, 2 0.8695, 4 0.8706, 8 0.8774 ms;
G = 4 became the default of both builders (graph.XCD_SLICE_GROUP). Each variant library builds
its own XCD plan (a fresh graph object per variant, the plans are cached per graph) and is timed
on the column-ordered graph as bench.py runs it.

    python tools/slice_group_ab.py --build [--groups 1,8,64]     (CPU side)
    python tools/slice_group_ab.py [--workload cfg2|ns] [--groups 1,8,64]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--groups", default="1,8,64")
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--snake", default="", help="group sizes dealt back and forth (variant sg<G>s)")
    a = ap.parse_args()
    groups = [int(v) for v in a.groups.split(",")]
    names = [f"sg{gsz}" for gsz in groups] + [f"sg{v}s" for v in a.snake.split(",") if v]
    if a.build:
        from graphneuralnetwork_amd.build import build_variant
        for gsz in groups:
            print(build_variant(f"sg{gsz}", [f"GNN_XCD_SLICE_GROUP={gsz}"], only=["plan_build.hip"]))
        for gsz in a.snake.split(","):
            if gsz:
                print(build_variant(f"sg{gsz}s", [f"GNN_XCD_SLICE_GROUP={gsz}", "GNN_XCD_SLICE_SNAKE"],
                                    only=["plan_build.hip"]))
        return
    import torch
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import column_order, spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, e = (1_000_000, 10_000_000) if a.workload == "cfg2" else (10_000_000, 100_000_000)
    s, d = rmat_edges(n, e, 0)
    F = a.feat
    g = column_order(gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n), F).graph
    X = torch.randn(n, F, device=dev)
    Y = torch.empty(n, F, device=dev)
    ref = spmm_forward(g, X).clone()
    graphs = {gsz: CsrGraph(g.rowptr, g.col, g.val, g.n_rows, g.n_cols) for gsz in names}
    times = {gsz: [] for gsz in names}
    for r in range(a.rounds):
        for gsz in names:
            _lib.use_variant(ROOT / "graphneuralnetwork_amd" / "lib" / "variants" / f"libgnn_{gsz}.so")
            gv = graphs[gsz]
            spmm_forward(gv, X, out=Y)
            torch.cuda.synchronize()
            if r == 0:
                err = float(((Y - ref).abs() / (ref.abs() + 1e-3)).max())
                print(json.dumps({"group": gsz, "max_rel_err_vs_default": err}), flush=True)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(5):
                spmm_forward(gv, X, out=Y)
            ev[1].record()
            torch.cuda.synchronize()
            times[gsz].append(ev[0].elapsed_time(ev[1]) / 5)
    print(json.dumps({"workload": a.workload, "feat": F,
                      "median_ms": {gsz: round(statistics.median(t), 4) for gsz, t in times.items()}}))


if __name__ == "__main__":
    main()
