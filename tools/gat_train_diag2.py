"""Per-stage diagnostics of the GAT backward at cfg3 against the float64 oracle run on the
GPU's own fp32 Wh: forward LSE stats, del, der, dWh, each with its worst rows.

    python tools/gat_train_diag2.py [--sparse] [--drop 0.0]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def worst(name, hip, ref, deg, k=8):
    e = np.abs(hip - ref)
    if e.ndim > 1:
        e = e.max(1)
        mag = np.abs(ref).max(1)
    else:
        mag = np.abs(ref)
    print(f"{name}: max err {e.max():.3e}, max |ref| {np.abs(ref).max():.3e}, "
          f"rows with err > 1e-4 max|ref| {(e > 1e-4 * np.abs(ref).max()).sum()}")
    for i in np.argsort(-e)[:k]:
        print(f"   row {i} deg {deg[i]} |ref| {mag[i]:.4g} err {e[i]:.4g}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sparse", action="store_true")
    ap.add_argument("--drop", type=float, default=0.0)
    a = ap.parse_args()
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    from oracle import c_oracle
    dev = torch.device("cuda:0")
    n, H, fh, Fin, seed = 1_000_000, 8, 8, 64, 0x5EED_0F_CF63
    mode = ops.GAT_SPARSE if a.sparse else ops.GAT_DENSE
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    gen = torch.Generator(dev).manual_seed(5)
    X = torch.randn(n, Fin, device=dev, generator=gen)
    W = torch.randn(Fin, H * fh, device=dev, generator=gen) * 0.25
    a_s = torch.randn(H * fh, device=dev, generator=gen) * 0.5
    a_d = torch.randn(H * fh, device=dev, generator=gen) * 0.5
    gy = torch.randn(n, H * fh, device=dev, generator=gen)
    wh = X @ W
    el, er = ops.gat_logits(wh, H, fh, a_s, a_d)
    stats = torch.empty((n, H), device=dev)
    y = ops.gat_aggregate(g, wh, el, er, H, fh, 0.2, mode, "elu", dropout_p=a.drop, seed=seed,
                          stats=stats, a_dst=a_d)
    dwh, dout, dl, der = ops.gat_backward(g, wh, el, er, stats, y, gy, a_s, a_d, H, fh, 0.2,
                                          mode, True, a.drop, seed)
    rowptr, col = g.rowptr.cpu().numpy(), g.col.cpu().numpy()
    deg = np.diff(rowptr)
    whn = wh.cpu().numpy().astype(np.float64)
    r = c_oracle.gat_block_grad(rowptr, col, whn, np.eye(H * fh), a_s.cpu().numpy(),
                                a_d.cpu().numpy(), gy.cpu().numpy(), H, fh, 0.2, a.sparse,
                                drop_p=a.drop, drop_seed=seed)
    # float64 LSE of the logits per (row, head)
    whh = whn.reshape(n, H, fh)
    el64 = (whh * a_s.cpu().numpy().astype(np.float64).reshape(H, fh)).sum(-1)
    er64 = (whh * a_d.cpu().numpy().astype(np.float64).reshape(H, fh)).sum(-1)
    row = np.repeat(np.arange(n), deg)
    t = el64[row] + er64[col]
    z = np.where(t > 0, t, 0.2 * t)
    if a.sparse:
        z = -z
    mx = np.maximum.reduceat(z, rowptr[:-1], axis=0)
    lse = mx + np.log(np.add.reduceat(np.exp(z - mx[row]), rowptr[:-1], axis=0))
    st = stats.cpu().numpy()
    worst("out", y.cpu().numpy(), r["out"], deg)
    worst("lse stats", st, lse, deg)
    worst("del", dl.cpu().numpy(), r["del"], deg)
    worst("der", der.cpu().numpy(), r["der"], deg)
    worst("dwh", dwh.cpu().numpy(), r["dwh"], deg)
    print("plan: seg_len", g.plan(ops.seg_len_for(H * fh, ops.GAT_SEG_BYTES)).seg_len,
          "short deg", ops.GAT_BWD_SHORT_DEG, "symmetric", g.symmetric)


if __name__ == "__main__":
    main()
