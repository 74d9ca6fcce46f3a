"""A/B of the fused GraphSAGE layer (ops.sage_layer, one launch) against the unfused
centre gather + gather-mean + hipBLASLt K=2F GEMM, on the cfg4 batch (RMAT 10M / 100M,
8192 seeds, fanout [25, 10], F = H = 128), layer 0 alone and the whole eval forward.

    python tools/sage_layer_ab.py [--rounds 8]
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
    ap.add_argument("--rounds", type=int, default=8)
    args = ap.parse_args()
    from graphneuralnetwork_amd import graphsage as GS
    from graphneuralnetwork_amd.ops import sage_layer
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import sample_batch, symmetric_adjacency
    dev = torch.device("cuda:0")
    n, F = 10_000_000, 128
    s, d = rmat_edges(n, 100_000_000, 0)
    adj = symmetric_adjacency(s, d, n, device=dev)
    del s, d
    gen = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(n, F, device=dev, generator=gen)
    deg = adj.rowptr[1:] - adj.rowptr[:-1]
    cand = torch.nonzero(deg > 0).view(-1)
    seeds = cand[torch.randperm(cand.numel(), device=dev, generator=gen)[:8192]]
    batch = sample_batch(adj, seeds, (25, 10), seed=0)
    net = GS.GraphSAGE(2, F, F, False, agg_func="MEAN", Unsupervised=False,
                       class_size=3).to(dev).eval()
    fargs = batch.forward_args(table)
    blk = net.sage_blocks.sage_layer0
    center = GS.Gathered(table, batch.frontier, True)
    neigh = GS.Gathered(table, batch.frontier_nbrs, True)
    real_sage_layer = GS.sage_layer

    def fused_on():
        GS.sage_layer = real_sage_layer

    def fused_off():
        GS.sage_layer = lambda *a, **kw: None

    def layer0():
        return GS._fused_sage_layer(blk, center, neigh)

    with torch.no_grad():
        h1 = layer0()
    blk1 = net.sage_blocks.sage_layer1
    c1 = GS.Gathered(h1, batch.center_map, True)
    n1 = GS.Gathered(h1, batch.neigh_map, True)

    def layer1():
        return GS._fused_sage_layer(blk1, c1, n1)

    def forward():
        return net(*fargs, None, None, None, None, None)

    nb1 = batch.frontier_nbrs[:, :1].contiguous()
    W0 = blk.weight.weight

    def layer0_k1():  # the fused kernel with one neighbour: ~ its MFMA phase + self gathers
        return real_sage_layer(table, nb1, W0, table, batch.frontier, check=False)

    buf = torch.randn(batch.frontier.numel(), 2 * F, device=dev)
    zero = torch.zeros(W0.shape[0], device=dev)

    def gemm0():  # the unfused path's hipBLASLt GEMM alone
        return torch._addmm_activation(zero, buf, W0.t())

    from graphneuralnetwork_amd import ops

    def forced():
        GS.sage_layer = real_sage_layer
        ops.SAGE_FUSED_MIN_ROWS = 1

    def default():
        GS.sage_layer = real_sage_layer
        ops.SAGE_FUSED_MIN_ROWS = min_rows

    min_rows = ops.SAGE_FUSED_MIN_ROWS
    fused_on = forced
    variants = {"layer0_fused_k1": (forced, layer0_k1), "gemm0_hipblaslt": (forced, gemm0),
                "layer1_fused": (forced, layer1), "layer1_unfused": (fused_off, layer1),
                "forward_default_policy": (default, forward),
                "layer0_fused": (fused_on, layer0), "layer0_unfused": (fused_off, layer0),
                "forward_fused": (fused_on, forward), "forward_unfused": (fused_off, forward)}
    with torch.no_grad():
        fused_on()
        a = layer0()
        fused_off()
        b = layer0()
        err = float((a - b).abs().max() / b.abs().max())
        assert err < 1e-5, err
        forced()
        assert real_sage_layer(table, batch.frontier_nbrs, blk.weight.weight, table,
                               batch.frontier, check=False) is not None
        # each variant replayed from a HIP graph of REP calls: GPU time, no Python pacing
        REP = 10
        graphs = {}
        for name, (setup, fn) in variants.items():
            setup()
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                fn()
                fn()
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(REP):
                    fn()
            graphs[name] = g
        times = {k: [] for k in variants}
        stream = torch.cuda.current_stream(dev)
        for _ in range(args.rounds):
            for name, g in graphs.items():
                g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                g.replay()
                e1.record(stream)
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / REP)
        default()
    M, k1 = batch.frontier_nbrs.shape
    print(json.dumps({"frontier": M, "k": k1, "seeds": int(seeds.numel()),
                      "sampled_edges": batch.sampled_edges, "layer0_max_rel_diff": err}), flush=True)
    for name, t in times.items():
        print(json.dumps({"variant": name, "median_us": round(statistics.median(t) * 1e3, 1),
                          "min_us": round(min(t) * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
