"""GAT inference layer at cfg3: projection outputs packed [Wh | er | el] in one buffer vs
three separate tensors (interleaved A/B, one process).

    python tools/gat_pack_ab.py
"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    from graphneuralnetwork_amd.ops import GAT_DENSE, gat_aggregate, gat_project
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n = 1_000_000
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n, device=dev)
    H, Fh, Fin = 8, 8, 64
    gen = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(n, Fin, device=dev, generator=gen)
    W = torch.randn(Fin, H * Fh, device=dev, generator=gen) * 0.2
    a_s = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    a_d = torch.randn(H * Fh, device=dev, generator=gen) * 0.3
    out = torch.empty(n, H * Fh, device=dev)
    proj = {p: gat_project(X, W, H, Fh, a_s, a_d, packed=p) for p in (False, True)}
    ref = gat_aggregate(g, *proj[False], H, Fh, 0.2, GAT_DENSE, "elu").clone()
    got = gat_aggregate(g, *proj[True], H, Fh, 0.2, GAT_DENSE, "elu")
    assert torch.equal(ref, got)
    fns = {}
    for p in (False, True):
        fns[f"layer_packed{int(p)}"] = (lambda p=p: gat_aggregate(
            g, *gat_project(X, W, H, Fh, a_s, a_d, packed=p), H, Fh, 0.2, GAT_DENSE, "elu",
            out=out))
        fns[f"agg_packed{int(p)}"] = (lambda p=p: gat_aggregate(
            g, *proj[p], H, Fh, 0.2, GAT_DENSE, "elu", out=out))
    t = {k: [] for k in fns}
    for _ in range(6):
        for k, f in fns.items():
            f()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                f()
            b.record()
            torch.cuda.synchronize()
            t[k].append(a.elapsed_time(b) / 5)
    print(json.dumps({k: statistics.median(v) for k, v in t.items()}), flush=True)


if __name__ == "__main__":
    main()
