"""The GAT models' F.dropout (GAT/models/GAT.py:15,17) in training as a hashed element mask
(ops.dropout_rows / DropoutRows / model_dropout, gnn_dropout_rows_f32), the first one fused
with the relabelling onto P A P^T: values and gradients bit-exact against the oracle's
restated mask (oracle_dropout_keep, the common.hpp dropout_hash over (seed, row, column)).
"""
import numpy as np
import pytest
import torch

from oracle import c_oracle

pytestmark = pytest.mark.gpu


def _expect(x, p, seed, rows, keys):
    """x[rows] with element (i, c) kept iff the (seed, keys[i], c) hash clears p, times
    float32(1 / (1 - p)) -- the kernel's arithmetic, in fp32."""
    F_ = x.shape[1]
    keep = c_oracle.dropout_keep(seed, keys[:, None], np.arange(F_)[None, :], p)
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    return np.where(keep, x[rows] * scale, np.float32(0.0)).astype(np.float32), keep


@pytest.mark.parametrize("feat", [64, 7, 128])
@pytest.mark.parametrize("gather", [False, True])
def test_dropout_rows_vs_oracle_mask(dev, feat, gather):
    from graphneuralnetwork_amd.ops import DropoutRows
    rng = np.random.default_rng(feat)
    n, p, seed = 5003, 0.4, 0x1234_5678_9abc_def
    x = rng.standard_normal((n, feat)).astype(np.float32)
    perm = rng.permutation(n) if gather else np.arange(n)
    inv = np.argsort(perm)
    xd = torch.from_numpy(x).to(dev).requires_grad_(True)
    pt = torch.from_numpy(perm).to(dev) if gather else None
    it = torch.from_numpy(inv).to(dev) if gather else None
    y = DropoutRows.apply(xd, p, seed, pt, it)
    want, keep = _expect(x, p, seed, perm, np.arange(n))
    np.testing.assert_array_equal(y.detach().cpu().numpy(), want)
    assert abs(1.0 - keep.mean() - p) < 0.02
    gy = rng.standard_normal((n, feat)).astype(np.float32)
    y.backward(torch.from_numpy(gy).to(dev))
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    gx = np.zeros_like(x)
    gx[perm] = np.where(keep, gy * scale, np.float32(0.0))
    np.testing.assert_array_equal(xd.grad.cpu().numpy(), gx)


def test_dropout_rows_strided_and_in_place_refused(dev):
    """A row-strided view (ldx > feat) takes the scalar path; in-place with a gather is refused."""
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import dropout_rows
    rng = np.random.default_rng(1)
    base = rng.standard_normal((300, 13)).astype(np.float32)
    xv = torch.from_numpy(base).to(dev)[:, 2:11]  # 9 columns, row pitch 13
    y = dropout_rows(xv, 0.3, 77)
    want, _ = _expect(base[:, 2:11], 0.3, 77, np.arange(300), np.arange(300))
    np.testing.assert_array_equal(y.cpu().numpy(), want)
    lib = _lib.load()
    t = torch.zeros((8, 4), device=dev)
    idx = torch.arange(8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = lib.gnn_dropout_rows_f32(t.data_ptr(), 4, 8, idx.data_ptr(), 0, 8, 4, 0.5, 1,
                                  t.data_ptr(), 4, err.data_ptr(), None)
    assert rc != 0
    rc = lib.gnn_dropout_rows_f32(t.data_ptr(), 4, 8, None, 0, 8, 4, 1.0, 1, t.data_ptr(), 4,
                                  err.data_ptr(), None)
    assert rc != 0  # p = 1 (torch returns zeros) is left to torch


def _gat_setup(dev, model, p, monkeypatch, fh=8):
    from graphneuralnetwork_amd import gat as gat_mod
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n, H, Fin, C = 20000, 4, 32, 7
    s, d = rmat_edges(n, 150_000, 3)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    order = ops.node_order(g)
    monkeypatch.setattr(gat_mod.GATBase, "_train_order", lambda self, x, adj: order)
    torch.manual_seed(0)
    net = getattr(gat_mod, model)(Fin, fh, C, p, 0.2, H).to(dev).train()
    # small inputs: SpGAT's exp(-LeakyReLU) weights overflow to inf / inf = NaN on large logits
    # (the reference's arithmetic and NaN assert, layers.py:102-124)
    X = (0.1 * torch.randn(n, Fin, device=dev)).requires_grad_(True)
    return gat_mod, ops, net, X, g, order


@pytest.mark.parametrize("model", ["GAT", "SpGAT"])
def test_gat_model_dropouts_vs_oracle_mask(dev, model, monkeypatch):
    """GATBase.forward in training over P A P^T with dropout 0.5, the hidden dropout unfused
    (GAT_FUSE_OUT_DROPOUT off): the heads' input is X[perm] under the oracle mask of the first
    seed, out_att's input the heads' output under the mask of the second, and X.grad is the
    heads' input gradient masked and scattered back through the permutation -- all bit-exact."""
    p = 0.5
    gat_mod, ops, net, X, g, order = _gat_setup(dev, model, p, monkeypatch)
    monkeypatch.setattr(gat_mod, "GAT_FUSE_OUT_DROPOUT", False)
    seeds, calls = [], []
    real_seed, real_md = ops.dropout_seed, gat_mod.model_dropout

    def rec_seed():
        seeds.append(real_seed())
        return seeds[-1]

    def rec_md(x, *a, **k):
        y = real_md(x, *a, **k)
        y.retain_grad()
        calls.append((x, y))
        return y
    monkeypatch.setattr(ops, "dropout_seed", rec_seed)
    monkeypatch.setattr(gat_mod, "model_dropout", rec_md)
    out = net(X, g)
    out.sum().backward()
    assert len(seeds) == 2 and len(calls) == 2
    n, Fin = X.shape
    perm = order.perm.cpu().numpy()
    want, keep = _expect(X.detach().cpu().numpy(), p, seeds[0], perm, np.arange(n))
    np.testing.assert_array_equal(calls[0][1].detach().cpu().numpy(), want)
    want2, _ = _expect(calls[1][0].detach().cpu().numpy(), p, seeds[1], np.arange(n),
                       np.arange(n))
    np.testing.assert_array_equal(calls[1][1].detach().cpu().numpy(), want2)
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    gx = np.zeros((n, Fin), np.float32)
    gx[perm] = np.where(keep, calls[0][1].grad.cpu().numpy() * scale, np.float32(0.0))
    np.testing.assert_array_equal(X.grad.cpu().numpy(), gx)


@pytest.mark.parametrize("fh", [8, 2])
@pytest.mark.parametrize("model", ["GAT", "SpGAT"])
def test_gat_model_fused_hidden_dropout_bit_identical(dev, model, fh, monkeypatch):
    """The hidden dropout inside the heads' op (its mask applied to dy by the backward prep,
    gnn_gat_backward_rows_ex_f32) gives the same bits as the separate pass (pinned above): the
    logits, X.grad and every parameter gradient, with the same seeds. fh = 2: the prep is fused
    into the row pass, rows_ex refuses the mask and dy is masked first (the fallback)."""
    p = 0.5
    gat_mod, ops, net, X, g, order = _gat_setup(dev, model, p, monkeypatch, fh)
    calls = []
    real = ops._gat_backward_recompute
    monkeypatch.setattr(ops, "_gat_backward_recompute",
                        lambda *a: calls.append(a[-1]) or real(*a))
    res = {}
    for fused in (False, True):
        monkeypatch.setattr(gat_mod, "GAT_FUSE_OUT_DROPOUT", fused)
        torch.manual_seed(11)
        X.grad = None
        net.zero_grad(set_to_none=True)
        out = net(X, g)
        out.backward(torch.ones_like(out) * 0.01)
        res[fused] = [out.detach().clone(), X.grad.clone()] + [q.grad.clone()
                                                               for q in net.parameters()]
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)
    assert any(c is not None for c in calls)  # the fused form ran (dy_dropout handed down)
