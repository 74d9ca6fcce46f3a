"""The cfg3 GAT aggregation (column-degree order, 8 x 8 heads, as bench.py run_gat) run a few
times with one library / er setting, for a PMC pass of one variant (rocprofv3 --pmc ...):

    python tools/gat_variant_run.py [--lib <variant tag>] [--rec] [--reps 5]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--rec", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from graphneuralnetwork_amd import _lib, ops
    from graphneuralnetwork_amd.build import LIB_DIR
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    if a.lib:
        _lib.use_variant(LIB_DIR / "variants" / f"libgnn_{a.lib}.so")
    ops.GAT_ER_RECOMPUTE = a.rec
    dev = torch.device("cuda:0")
    s, d = rmat_edges(1_000_000, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), 1_000_000, device=dev)
    H, Fh, Fin = 8, 8, 64
    gen = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(g.n_rows, Fin, device=dev, generator=gen)
    W = torch.randn(Fin, H * Fh, device=dev, generator=gen) * 0.2
    a_s = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    a_d = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    order = ops.gat_column_order(g, H, Fh)
    wh, el, er = ops.gat_project(X, W, H, Fh, a_s, a_d, col_rows=order.inv)
    out = torch.empty_like(wh)
    for _ in range(a.reps):
        ops.gat_aggregate(order.graph, wh, el, er, H, Fh, 0.2, ops.GAT_DENSE, "elu", out=out,
                          a_dst=a_d)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
