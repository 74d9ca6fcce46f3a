"""Interleaved A/B of the cfg4 GraphSAGE forward (8192 seeds, [25, 10], 10M / 100M R-MAT,
F=H=128, eval; the degree-ordered dataset as bench.py) with the SageLayer GEMMs on hipBLASLt
vs the hand-written fp32-MFMA kernel (graphsage._sage_gemm_on_mfma; the last layer's MFMA GEMM
carries the classifier epilogue), eager and replayed from a HIP graph.

    python tools/sage_gemm_forward_ab.py [--rounds 8]
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
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import degree_ordered, sample_batch, symmetric_adjacency
    dev = torch.device("cuda:0")
    n, F = 10_000_000, 128
    s, d = rmat_edges(n, 100_000_000, 0)
    adj, _, _ = degree_ordered(symmetric_adjacency(s, d, n, device=dev))  # as bench.py
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
    default = GS._sage_gemm_on_mfma
    policies = {"hipblaslt": lambda rows: False, "mfma all": lambda rows: True,
                "mfma small": lambda rows: rows <= 16384 or rows >= 131072,
                "default": default}
    outs, graphs = {}, {}
    with torch.no_grad():
        for name, pol in policies.items():
            GS._sage_gemm_on_mfma = pol
            outs[name] = net(*fargs, None, None, None, None, None)[1].clone()
            s_cap = torch.cuda.Stream(dev)
            s_cap.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s_cap):
                net(*fargs, None, None, None, None, None)
            torch.cuda.current_stream(dev).wait_stream(s_cap)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                net(*fargs, None, None, None, None, None)
            graphs[name] = g
        ref = outs["hipblaslt"]
        times = {f"{k} {m}": [] for k in policies for m in ("eager", "graph")}
        for _ in range(args.rounds):
            for name, pol in policies.items():
                GS._sage_gemm_on_mfma = pol
                for mode, fn in (("eager", lambda: net(*fargs, None, None, None, None, None)),
                                 ("graph", graphs[name].replay)):
                    fn()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(10):
                        fn()
                    b.record()
                    torch.cuda.synchronize()
                    times[f"{name} {mode}"].append(a.elapsed_time(b) / 10)
        GS._sage_gemm_on_mfma = default
    print(json.dumps({"frontier": int(batch.frontier_nbrs.shape[0]), "seeds": 8192,
                      "max_rel_err_vs_hipblaslt": {
                          k: float((v - ref).abs().max() / ref.abs().max()) for k, v in outs.items()}}))
    for k, v in times.items():
        print(json.dumps({"variant": k, "median_us": round(statistics.median(v) * 1e3, 2),
                          "min_us": round(min(v) * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
