"""Interleaved A/B of GAT aggregation builds (lib/variants/*.so) at cfg3 (one process).

    python tools/gat_ab.py --variants base,j1,... [--rounds 6]
Variants are built on the CPU side by ``python tools/gat_ab.py --build`` (see VARIANTS).
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

# Measured and not kept (profiles/r02x_gat_pipe2.log): a depth-2 chunk pipeline (chunk
# k+1's er / Wh loads in flight while chunk k is reduced, two register buffers) -- 0.98 ms
# against 0.80: 84 VGPRs (5 waves/SIMD) cost more than the deeper pipeline gains.
# Also measured and not kept (round 4, profiles/r04gs_gat_short_rows_per_group_ab.log, --ordered):
# gat_short_kernel with RPG = 2 / 3 / 4 rows per lane group, their chains issued together:
# 0.809 / 0.837 / 0.883 ms against 0.783 at one row per group (RPG 2 + short chunk 8: 0.839).
VARIANTS = {
    "j1u2": ["GNN_GAT_CHUNK=1", "GNN_GAT_U=2"],     # one pass per chunk (previous kernel)
    "c32u2": ["GNN_GAT_CHUNK=32", "GNN_GAT_U=2"],
    "c32u4": ["GNN_GAT_CHUNK=32", "GNN_GAT_U=4"],
    "c64u4": ["GNN_GAT_CHUNK=64", "GNN_GAT_U=4"],
    "c16u2": ["GNN_GAT_CHUNK=16", "GNN_GAT_U=2"],
    "c16u2w8": ["GNN_GAT_CHUNK=16", "GNN_GAT_U=2", "GNN_GAT_WAVES_PER_EU=8"],
    "c8u2": ["GNN_GAT_CHUNK=8", "GNN_GAT_U=2"],
    "nopipe": ["GNN_GAT_PIPE=0"],
    "pipe": ["GNN_GAT_PIPE=1"],
    "base": [],
    "gs8": ["GNN_GAT_SMALL_UNROLL=8"],
    "gs16": ["GNN_GAT_SMALL_UNROLL=16"],
    "gs4": ["GNN_GAT_SMALL_UNROLL=4"],
    "gs2": ["GNN_GAT_SMALL_UNROLL=2"],
    "c16": ["GNN_GAT_CHUNK=16"],
    "c32": ["GNN_GAT_CHUNK=32"],
    "u2": ["GNN_GAT_U=2"],
    "gs4u4": ["GNN_GAT_SMALL_UNROLL=4", "GNN_GAT_U=4"],
    "gs4c16": ["GNN_GAT_SMALL_UNROLL=4", "GNN_GAT_CHUNK=16"],
    "gs4c16u4": ["GNN_GAT_SMALL_UNROLL=4", "GNN_GAT_CHUNK=16", "GNN_GAT_U=4"],
    "gs4np": ["GNN_GAT_SMALL_UNROLL=4", "GNN_GAT_PIPE=0"],
    "sc4": ["GNN_GAT_SHORT_CHUNK=4"],
    "sc16": ["GNN_GAT_SHORT_CHUNK=16"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--ordered", action="store_true",
                    help="the column-ordered graph with Wh / er rows in that order, as bench.py")
    ap.add_argument("--short-degs", default="",
                    help="instead of library variants: time the default build with these "
                         "GAT_SHORT_MAX_DEG values (0 = short-row path off)")
    args = ap.parse_args()
    names = args.variants.split(",")
    if args.build:
        from graphneuralnetwork_amd.build import build_variant
        for n in names:
            print(build_variant(n, VARIANTS[n], only=["gat.hip"]))
        return
    import torch
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import GAT_DENSE, gat_aggregate, gat_logits
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n = 1_000_000
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n, device=dev)
    H, Fh = 8, 8
    gen = torch.Generator(device=dev).manual_seed(0)
    Wh = torch.randn(n, H * Fh, device=dev, generator=gen)
    a_s = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    a_d = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    el, er = gat_logits(Wh, H, Fh, a_s, a_d)
    if args.ordered:
        from graphneuralnetwork_amd.ops import gat_column_order
        o = gat_column_order(g, H, Fh)
        g, Wh, er = o.graph, Wh[o.perm].contiguous(), er[o.perm].contiguous()
    out = torch.empty_like(Wh)
    from graphneuralnetwork_amd import ops as _ops
    _deg, _ops.GAT_SHORT_MAX_DEG = _ops.GAT_SHORT_MAX_DEG, 0
    ref = gat_aggregate(g, Wh, el, er, H, Fh, 0.2, GAT_DENSE, "elu").clone()  # short path off
    _ops.GAT_SHORT_MAX_DEG = _deg
    from graphneuralnetwork_amd import ops
    if args.short_degs:
        names = [f"short{d}" for d in args.short_degs.split(",")]
        libs = {v: None for v in names}
    else:
        libs = {v: ROOT / "graphneuralnetwork_amd" / "lib" / "variants" / f"libgnn_{v}.so"
                for v in names}
    times = {v: [] for v in names}
    for r in range(args.rounds):
        for v in names:
            if args.short_degs:
                ops.GAT_SHORT_MAX_DEG = int(v[5:])
            else:
                _lib.use_variant(libs[v])
            f = lambda: gat_aggregate(g, Wh, el, er, H, Fh, 0.2, GAT_DENSE, "elu", out=out)  # noqa
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                f()
            b.record()
            torch.cuda.synchronize()
            times[v].append(a.elapsed_time(b) / 10)
            if r == 0:
                err = (out - ref).abs().max().item()
                print(f"{v}: max |diff| vs the one-row-per-wave path {err:.3g}", flush=True)
    bytes_agg = g.nnz * (4 + 4 * H + 4 * H * Fh) + n * (8 + 4 * H + 4 * H * Fh)
    res = {v: {"ms": statistics.median(t), "GBps": bytes_agg / statistics.median(t) / 1e6}
           for v, t in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
