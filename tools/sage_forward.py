"""cfg4 GraphSAGE forward only (for rocprofv3 kernel breakdowns):

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python tools/sage_forward.py
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main(steps=20):
    from graphneuralnetwork_amd.graphsage import GraphSAGE
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
    net = GraphSAGE(2, F, F, False, agg_func="MEAN", Unsupervised=False, class_size=3).to(dev).eval()
    fargs = batch.forward_args(table)
    torch.cuda.synchronize()
    with torch.no_grad():
        for _ in range(steps):
            net(*fargs, None, None, None, None, None)
    torch.cuda.synchronize()
    print("frontier", batch.frontier.numel(), "sampled edges", batch.sampled_edges)


if __name__ == "__main__":
    main()
