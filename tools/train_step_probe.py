"""The benchmarked training steps alone, for a kernel trace (rocprofv3 --kernel-trace --stats):
the cfg2 Graph_conv_layer(128, 128) step (X requiring grad) or the cfg3 8 x 8-head GAT block
step (W, a_src, a_dst requiring grad), as bench.py's gcn_train_step / gat_train_step (over the
degree-ordered graph P A P^T the models train on, unless --natural); prints the HIP-event
median step time.

    python tools/train_step_probe.py --model gcn|gat [--steps 10] [--er-gather]
"""
from __future__ import annotations

import argparse
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=("gcn", "gat", "gcn_model", "gat_model"), default="gcn")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--er-gather", action="store_true",
                    help="GAT: er loaded, not recomputed from the gathered rows")
    ap.add_argument("--natural", action="store_true",
                    help="the natural-order graph (default: P A P^T, as the models train)")
    ap.add_argument("--set", action="append", default=[],
                    help="NAME=0|1: an ops switch (e.g. GCN_OVERLAP_DW=0)")
    a = ap.parse_args()
    for kv in a.set:
        from graphneuralnetwork_amd import ops
        k, v = kv.split("=")
        assert hasattr(ops, k), k
        setattr(ops, k, bool(int(v)))
    if a.er_gather:
        from graphneuralnetwork_amd import ops
        ops.GAT_ER_RECOMPUTE = False
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, m = (1_000_000, 10_000_000)
    s, d = rmat_edges(n, m, 0)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), n, device=dev)
    gen = torch.Generator(device=dev).manual_seed(1)
    from graphneuralnetwork_amd.ops import gat_train_order, gcn_train_order
    if a.model.endswith("_model"):  # the whole model, x and the logits in the original order
        if a.natural:
            from graphneuralnetwork_amd import ops
            ops.GCN_TRAIN_ORDER = ops.GAT_TRAIN_ORDER = False
        if a.model == "gcn_model":
            from graphneuralnetwork_amd.gcn import GCN_Model
            net = GCN_Model(128, 128, 7, 2, 0.5).to(dev).train()
            X = torch.randn(n, 128, device=dev, generator=gen)
        else:
            from graphneuralnetwork_amd.gat import GAT
            net = GAT(64, 8, 7, dropout=0.6, alpha=0.2, nheads=8).to(dev).train()
            X = torch.randn(n, 64, device=dev, generator=gen)
        labels = torch.randint(0, 7, (n,), device=dev, generator=gen)
        idx_train = torch.arange(0, n, 10, device=dev)
        ce = torch.nn.CrossEntropyLoss()

        def step():  # the reference loops: CE on output[idx_train] (GCN/train_eval.py:43-46)
            net.zero_grad(set_to_none=True)
            ce(net(X, g)[idx_train], labels[idx_train]).backward()
    elif not a.natural:
        o = gcn_train_order(g, 128) if a.model == "gcn" else gat_train_order(g, 8, 8)
        g = o.graph if o is not None else g
    if a.model.endswith("_model"):
        pass
    elif a.model == "gcn":
        from graphneuralnetwork_amd.gcn import Graph_conv_layer
        net = Graph_conv_layer(128, 128).to(dev)
        X = torch.randn(n, 128, device=dev, generator=gen).requires_grad_(True)
        gy = torch.randn(n, 128, device=dev, generator=gen)

        def step():
            X.grad = None
            net.zero_grad(set_to_none=True)
            net(X, g).backward(gy)
    else:
        from graphneuralnetwork_amd.gat import GAT
        net = GAT(64, 8, 3, dropout=0.0, alpha=0.2, nheads=8).to(dev).train()
        X = torch.randn(n, 64, device=dev, generator=gen)
        gy = torch.randn(n, 64, device=dev, generator=gen)

        def step():
            net.zero_grad(set_to_none=True)
            net._heads(X, g).backward(gy)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        step()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"{a.model} train step median {statistics.median(ts):.4f} ms over {a.steps}", flush=True)


if __name__ == "__main__":
    main()
