"""Diagnostics for the full-size GAT training pin (tests/test_fullsize_gpu.py): where the HIP
block gradients differ from the float64 oracle, and how much the oracle itself moves when its
Wh is rounded to fp32 (the conditioning of each gradient at this graph).

    python tools/gat_train_diag.py [--model GAT|SpGAT] [--drop 0.0]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="SpGAT")
    ap.add_argument("--drop", type=float, default=0.0)
    a = ap.parse_args()
    from graphneuralnetwork_amd import gat as gat_mod
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    from oracle import c_oracle
    dev = torch.device("cuda:0")
    n, H, fh, Fin, seed = 1_000_000, 8, 8, 64, 0x5EED_0F_CF63
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    torch.manual_seed(1)
    net = getattr(gat_mod, a.model)(Fin, fh, 7, a.drop, 0.2, H).to(dev).train()
    gat_mod._dropout_seed = lambda: seed
    gen = torch.Generator(dev).manual_seed(5)
    X = torch.randn(n, Fin, device=dev, generator=gen).requires_grad_(True)
    gy = torch.randn(n, H * fh, device=dev, generator=gen)
    out = net._heads(X, g)
    out.backward(gy)
    W = torch.cat([m.W for m in net.attentions], 1).detach().cpu().numpy()
    av = [m.a.detach().reshape(-1).cpu().numpy() for m in net.attentions]
    a_s = np.concatenate([x[:fh] for x in av])
    a_d = np.concatenate([x[fh:] for x in av])
    rowptr, col = g.rowptr.cpu().numpy(), g.col.cpu().numpy()
    deg = np.diff(rowptr)
    Xn = X.detach().cpu().numpy()
    gyn = gy.cpu().numpy()
    r = c_oracle.gat_block_grad(rowptr, col, Xn, W, a_s, a_d, gyn, H, fh, 0.2,
                                a.model == "SpGAT", drop_p=a.drop, drop_seed=seed)
    # the oracle on Wh rounded to fp32 (x W in float64, stored as fp32 -- what any fp32
    # implementation holds): its distance from the exact oracle is the gradients' conditioning
    wh32 = (Xn.astype(np.float64) @ W.astype(np.float64)).astype(np.float32)
    r32 = c_oracle.gat_block_grad(rowptr, col, wh32.astype(np.float64), np.eye(H * fh), a_s,
                                  a_d, gyn, H, fh, 0.2, a.model == "SpGAT", drop_p=a.drop,
                                  drop_seed=seed)  # x = Wh32, W = I: the oracle on fp32 Wh
    dx = X.grad.cpu().numpy()
    for k, hip, ref, ref32 in (("out", out.detach().cpu().numpy(), r["out"], r32["out"]),
                               ("dwh->dx", dx, r["dx"], r32["dwh"] @ W.astype(np.float64).T)):
        e = np.abs(hip - ref)
        e32 = np.abs(ref32 - ref)
        print(f"{k}: max|hip-ref|/max|ref| {e.max() / np.abs(ref).max():.3e}; "
              f"max|ref32-ref|/max|ref| {e32.max() / np.abs(ref).max():.3e}")
        rows = np.argsort(-e.max(1))[:12]
        for i in rows:
            print(f"  row {i} deg {deg[i]} max|ref row| {np.abs(ref[i]).max():.4g} "
                  f"err {e[i].max():.4g} ref32 err {e32[i].max():.4g}")
    print("hub degrees", deg[np.argsort(-deg)[:5]])


if __name__ == "__main__":
    main()
