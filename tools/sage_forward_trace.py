"""Runs the cfg4 GraphSAGE forward (degree-ordered dataset, 8192 seeds, [25, 10]) REPS times
after warm-up, for a rocprofv3 --kernel-trace of its kernels:

    rocprofv3 --kernel-trace -d gpurun_out/sage_trace -o run -- python3 tools/sage_forward_trace.py
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import degree_ordered, sample_batch, symmetric_adjacency
    dev = torch.device("cuda:0")
    n, F = 10_000_000, 128
    s, d = rmat_edges(n, 100_000_000, 0)
    adj, _, _ = degree_ordered(symmetric_adjacency(s, d, n, device=dev))
    del s, d
    gen = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(n, F, device=dev, generator=gen)
    deg = adj.rowptr[1:] - adj.rowptr[:-1]
    cand = torch.nonzero(deg > 0).view(-1)
    seeds = cand[torch.randperm(cand.numel(), device=dev, generator=gen)[:8192]]
    b = sample_batch(adj, seeds, (25, 10), seed=0)
    net = GraphSAGE(2, F, F, False, agg_func="MEAN", Unsupervised=False, class_size=3).to(dev).eval()
    fa = b.forward_args(table)
    with torch.no_grad():
        for _ in range(10):
            net(*fa, None, None, None, None, None)
        torch.cuda.synchronize()
        torch.cuda.nvtx.range_push("forwards") if hasattr(torch.cuda, "nvtx") else None
        for _ in range(50):
            net(*fa, None, None, None, None, None)
        torch.cuda.synchronize()
    print("done", b.frontier.numel())


if __name__ == "__main__":
    main()
