"""Interleaved A/B of whole-library builds (lib/variants/libgnn_<tag>.so, built by
build.build_variant) on the default SpMM path (ops.spmm_forward) at one workload.

    python tools/lib_ab.py --build --variants base,ntcold      (CPU side)
    python tools/lib_ab.py --variants base,ntcold [--workload cfg2|ns] [--feat 128]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

# tag -> -D flags. Variant libraries export only the C-ABI (build.EXPORT_MAP), so each
# one launches its own kernels; before round 2 they did not (the kernels' weak template
# symbols bound to the main library), and every round-1 library A/B compared the main
# build with itself.
# Non-temporal loads for the cold (non-hub) gathers, so they leave the hub rows in L2:
# no change (cfg2 1.134 vs 1.136 ms, ns 14.37 vs 14.37 ms, profiles/r02q_nt_*.log).
# Prefetching the next 64-edge (col, val) chunk during the current one: no change (cfg2
# 1.133 vs 1.134 ms, ns 14.21 vs 14.23 ms, profiles/r02o_pf_*.log), not kept.
# Short rows (2..16 edges) in their own launch, 64/LPS rows per wave (LPS lanes x 4 16-B
# chunks, 2 edges in flight per lane): slower at every threshold (cfg2 1.136 ms off, 1.144
# at <= 4, 1.168 at <= 16, 1.211 at <= 64; ns 14.35 off vs 14.41), profiles/r02p_short_*.log;
# not kept: the one-wave-per-row mid path already overlaps those rows' latency.
# GCN transform grid (tools/transform_ab.py --variants, profiles/r02m_transform_ab.log):
# 512 workgroups 0.300 ms at 1M x 128 x 128, 256: 0.333, 768: 0.316, 1024: 0.30x.
VARIANTS = {
    "base": [],
    "tu2": ["GNN_SPMM_TASK_U=2"],
    "tu8": ["GNN_SPMM_TASK_U=8"],
    "tu16": ["GNN_SPMM_TASK_U=16"],
    "tf256": ["GNN_TF_GRID=256"],
    "tf768": ["GNN_TF_GRID=768"],
    "tf1024": ["GNN_TF_GRID=1024"],
    "u2": ["GNN_SPMM_U=2"],
    "u8": ["GNN_SPMM_U=8"],
    "small2": ["GNN_SPMM_SMALL_UNROLL=2"],
    "small8": ["GNN_SPMM_SMALL_UNROLL=8"],
    "small16": ["GNN_SPMM_SMALL_UNROLL=16"],
    "split8": ["GNN_SPMM_SMALL_SPLIT=1", "GNN_SPMM_SMALL_SPLIT_UNROLL=8"],
    "split16": ["GNN_SPMM_SMALL_SPLIT=1", "GNN_SPMM_SMALL_SPLIT_UNROLL=16"],
    "split32": ["GNN_SPMM_SMALL_SPLIT=1", "GNN_SPMM_SMALL_SPLIT_UNROLL=32"],
    # occupancy caps by dynamic LDS (160 KiB per CU): at most 6 / 4 / 3 / 2 workgroups per CU
    "wg6": ["GNN_SPMM_LDS_PAD=26624", "GNN_GAT_LDS_PAD=26624", "GNN_SAGE_LDS_PAD=26624"],
    "wg4": ["GNN_SPMM_LDS_PAD=40960", "GNN_GAT_LDS_PAD=40960", "GNN_SAGE_LDS_PAD=40960"],
    "wg3": ["GNN_SPMM_LDS_PAD=53248", "GNN_GAT_LDS_PAD=53248", "GNN_SAGE_LDS_PAD=53248"],
    "wg2": ["GNN_SPMM_LDS_PAD=65536", "GNN_GAT_LDS_PAD=65536", "GNN_SAGE_LDS_PAD=65536"],
    "s16u8": ["GNN_SPMM_SMALL_UNROLL=16", "GNN_SPMM_U=8"],
    "s16u2": ["GNN_SPMM_SMALL_UNROLL=16", "GNN_SPMM_U=2"],
    "small32": ["GNN_SPMM_SMALL_UNROLL=32"],
    "small4": ["GNN_SPMM_SMALL_UNROLL=4"],
    "s2": ["GNN_SPMM_SMALL_UNROLL=2"],
    "s4u8": ["GNN_SPMM_SMALL_UNROLL=4", "GNN_SPMM_U=8"],
    "s2u8": ["GNN_SPMM_SMALL_UNROLL=2", "GNN_SPMM_U=8"],
    "s4u6": ["GNN_SPMM_SMALL_UNROLL=4", "GNN_SPMM_U=6"],
    "s4u12": ["GNN_SPMM_SMALL_UNROLL=4", "GNN_SPMM_U=12"],
    "s4u16": ["GNN_SPMM_SMALL_UNROLL=4", "GNN_SPMM_U=16"],
    "sp4u8": ["GNN_SPMM_SMALL_SPLIT=1", "GNN_SPMM_SMALL_SPLIT_UNROLL=4", "GNN_SPMM_U=8"],
    "sp8u8": ["GNN_SPMM_SMALL_SPLIT=1", "GNN_SPMM_SMALL_SPLIT_UNROLL=8", "GNN_SPMM_U=8"],
    "sp16u8": ["GNN_SPMM_SMALL_SPLIT=1", "GNN_SPMM_SMALL_SPLIT_UNROLL=16", "GNN_SPMM_U=8"],
    "su2": ["GNN_SAGE_U=2"],
    "su8": ["GNN_SAGE_U=8"],
    "su16": ["GNN_SAGE_U=16"],
    "su4": ["GNN_SAGE_U=4"],
    # edge (col, val) moved to the edge slots by v_readlane + select instead of ds_bpermute:
    # slower (cfg2 0.946 vs 0.870 ms, ns 11.87 vs 11.79 ms, profiles/r05u_readlane_*.log)
    "readlane": ["GNN_SPMM_READLANE=1"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--only", default="spmm.hip,sage.hip",
                    help="--build: csrc files compiled with the variant's defines (the rest "
                         "link from the main build)")
    ap.add_argument("--seg-lens", default="", help="also time the default build at these seg_len")
    ap.add_argument("--ordered", action="store_true",
                    help="time the column-ordered graph A P^T, as bench.py does")
    ap.add_argument("--op", default="spmm", choices=["spmm", "sage"],
                    help="sage: the fused gather-mean over [M=62,401, k=10] uniform-degree-weighted "
                         "samples of the workload's graph (the cfg4 layer-0 shape)")
    args = ap.parse_args()
    names = args.variants.split(",")  # "tag" or "tag@seg_len"
    if args.build:
        from graphneuralnetwork_amd.build import build_variant
        for n in {n.split("@")[0] for n in names}:
            print(build_variant(n, VARIANTS[n], only=[f for f in args.only.split(",") if f]))
        return
    import torch
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, e = (1_000_000, 10_000_000) if args.workload == "cfg2" else (10_000_000, 100_000_000)
    s, d = rmat_edges(n, e, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n, device=dev)
    F = args.feat
    if args.ordered:
        from graphneuralnetwork_amd.ops import column_order
        o = column_order(g, F)
        g = g if o is None else o.graph
    X = torch.randn(n, F, device=dev)
    Y = torch.empty(n, F, device=dev)
    nbytes = g.nnz * (8 + 4 * F) + n * (8 + 4 * F)
    if args.op == "sage":
        from graphneuralnetwork_amd.ops import sage_gather_aggregate
        from graphneuralnetwork_amd.sampler import sample_neighbors
        deg = g.rowptr[1:] - g.rowptr[:-1]
        cand = torch.nonzero(deg > 0).view(-1)
        nodes = cand[torch.randperm(cand.numel(), device=dev)[:62401]]
        idx = sample_neighbors(g, nodes, 10, 0)
        Y = torch.empty(idx.shape[0], F, device=dev)
        nbytes = idx.numel() * (4 * F + 8) + idx.shape[0] * 4 * F

        def spmm_forward(g_, X_, out=None, seg_len=None):  # noqa: F811 -- same harness
            return sage_gather_aggregate(X_, idx, "MEAN", check=False, out=out)
    ref = spmm_forward(g, X, out=torch.empty_like(Y)).clone()
    libs = {v: ROOT / "graphneuralnetwork_amd" / "lib" / "variants" /
            f"libgnn_{v.split('@')[0]}.so" for v in names}
    seg = {v: int(v.split("@")[1]) for v in names if "@" in v}
    seg.update({f"seg{sl}": int(sl) for sl in args.seg_lens.split(",") if sl})
    names = names + [k for k in seg if k not in names]
    times = {v: [] for v in names}
    for r in range(args.rounds):
        for v in names:
            _lib.use_variant(libs[v] if v in libs and libs[v].exists() else None)
            sl = seg.get(v)
            spmm_forward(g, X, out=Y, seg_len=sl)
            torch.cuda.synchronize()
            if r == 0 and sl is None:
                assert torch.equal(Y, ref), v
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20 if args.op == "sage" else 5):
                spmm_forward(g, X, out=Y, seg_len=sl)
            b.record()
            torch.cuda.synchronize()
            times[v].append(a.elapsed_time(b) / (20 if args.op == "sage" else 5))
    for v, t in times.items():
        m = statistics.median(t)
        print(json.dumps({"variant": v, "op": args.op, "workload": args.workload, "feat": F, "median_ms": m,
                          "algo_GBps": nbytes / m / 1e6}), flush=True)


if __name__ == "__main__":
    main()
