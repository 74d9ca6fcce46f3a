"""Training path of Graph_conv_layer (GCN/GCN.py:41-47 under GCN/train_eval.py:43-48's
loss.backward()): ops.gcn_layer / _GcnLayerFn against float64 references.

Tolerance (north_star): fp32 within 1e-4 relative (atol scaled by max |ref|).
"""
import numpy as np
import pytest
import torch

from oracle import c_oracle

pytestmark = pytest.mark.gpu
RTOL = 1e-4


def close(a, b, rtol=RTOL):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(1.0, float(np.nanmax(np.abs(b)))) if b.size else 1.0
    np.testing.assert_allclose(a, b, rtol=rtol, atol=1e-5 * scale)


def _rand_graph(n, m, seed):
    rng = np.random.default_rng(seed)
    r = rng.integers(0, n, m)
    c = np.where(rng.random(m) < 0.3, rng.integers(0, 8, m), rng.integers(0, n, m))
    order = np.lexsort((c, r))
    r, c = r[order], c[order]
    rowptr = np.zeros(n + 1, np.int64)
    np.add.at(rowptr, r + 1, 1)
    return np.cumsum(rowptr), c.astype(np.int32), rng.standard_normal(m).astype(np.float32)


@pytest.mark.parametrize("fout", [7, 64, 128])
@pytest.mark.parametrize("bias", [True, False])
def test_gcn_layer_grads_vs_float64(dev, bias, fout):
    """A non-symmetric graph (transposed CSR built for dX): Y, dX, dW, db against float64
    dense autograd of A (X W^T) + b, in both of _GcnLayerFn's forms (128 -> 64: A (X W^T);
    128 -> 128: (A X) W^T, ops.GCN_REASSOC; 128 -> 7: A (X W^T) zero-padded to 8 columns,
    ops.GCN_PAD_NARROW)."""
    from graphneuralnetwork_amd.gcn import Graph_conv_layer
    from graphneuralnetwork_amd.graph import CsrGraph
    n = 400
    rowptr, col, val = _rand_graph(n, 5000, 3)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.from_numpy(val).to(dev), n, n)
    A = torch.zeros(n, n, dtype=torch.float64)
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    A.index_put_((torch.from_numpy(rows), torch.from_numpy(col.astype(np.int64))),
                 torch.from_numpy(val.astype(np.float64)), accumulate=True)
    layer = Graph_conv_layer(128, fout, is_bias=bias).to(dev)
    if bias:
        torch.nn.init.normal_(layer.bias)
    X = torch.randn(n, 128, device=dev, requires_grad=True)
    y = layer(X, g)
    gy = torch.randn_like(y)
    y.backward(gy)
    assert not g.symmetric and g._transpose is not None
    Xd = X.detach().cpu().double().requires_grad_()
    Wd = layer.dense.weight.detach().cpu().double().requires_grad_()
    bd = layer.bias.detach().cpu().double().requires_grad_() if bias else None
    yd = A @ (Xd @ Wd.t()) + (bd if bias else 0)
    yd.backward(gy.cpu().double())
    close(y.detach().cpu().numpy(), yd.detach().numpy())
    close(X.grad.cpu().numpy(), Xd.grad.numpy())
    close(layer.dense.weight.grad.cpu().numpy(), Wd.grad.numpy())
    if bias:
        close(layer.bias.grad.cpu().numpy(), bd.grad.numpy())


@pytest.mark.parametrize("fin,fout", [(128, 128), (64, 128), (128, 64), (128, 256)])
@pytest.mark.parametrize("x_grad", [True, False])
def test_gcn_layer_forms_agree(dev, fin, fout, x_grad, monkeypatch):
    """_GcnLayerFn's two forms of one layer -- A (X W^T) + b and (A X) W^T + b (GCN_REASSOC,
    taken when in_features <= out_features) -- give the same output and gradients to fp32
    rounding, with and without dX; the reassociated backward with X needing no gradient runs
    no SpMM (its dW = dY^T Z needs Z = A X from the forward only)."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.gcn import Graph_conv_layer
    from graphneuralnetwork_amd.graph import CsrGraph
    rp, col, val = _rand_graph(3000, 30000, 4)
    g = CsrGraph(torch.from_numpy(rp).to(dev), torch.from_numpy(col).to(dev),
                 torch.from_numpy(val).to(dev), 3000, 3000)
    torch.manual_seed(fin + fout)
    layer = Graph_conv_layer(fin, fout).to(dev)
    with torch.no_grad():
        layer.bias.normal_()
    X = torch.randn(3000, fin, device=dev)
    gy = torch.randn(3000, fout, device=dev)
    calls = []
    real = ops.spmm_forward
    monkeypatch.setattr(ops, "spmm_forward", lambda *a, **k: calls.append(1) or real(*a, **k))
    res = {}
    for re in (True, False):
        monkeypatch.setattr(ops, "GCN_REASSOC", re)
        assert ops._reassociate(X, layer.dense.weight, g) == (re and fin <= fout)
        xx = X.clone().requires_grad_(x_grad)
        layer.zero_grad(set_to_none=True)
        calls.clear()
        y = layer(xx, g)
        n_fwd = len(calls)
        y.backward(gy)
        n_bwd = len(calls) - n_fwd
        if re and fin <= fout and not x_grad:
            assert n_bwd == 0  # dW = dY^T Z, db = colsum dY: no SpMM
        else:
            assert n_bwd == 1
        res[re] = [y.detach(), layer.dense.weight.grad, layer.bias.grad] + (
            [xx.grad] if x_grad else [])
    for a, b in zip(res[True], res[False]):
        close(a.cpu().numpy(), b.cpu().numpy())


def test_transform_bias_and_tn_dsum_of_b(dev):
    """gnn_gcn_transform_bias_f32: x W^T + b equals the transform plus b to fp32 rounding of
    the one add (bit for bit), at 128 -> 128 and the split 256 -> 256; gnn_gemm_tn_f32 with
    d == b (the x6 kernel's DB form: dsum from B's own loads) equals the three-operand call
    with a copy of B as D, bit for bit."""
    from graphneuralnetwork_amd.ops import gcn_transform, gemm_tn
    gen = torch.Generator(device=dev).manual_seed(9)
    for k, fo, n in ((128, 128, 50001), (256, 256, 7000), (64, 64, 333)):
        x = torch.randn(n, k, device=dev, generator=gen)
        w = torch.randn(fo, k, device=dev, generator=gen)
        b = torch.randn(fo, device=dev, generator=gen)
        y0 = gcn_transform(x, w)
        y1 = gcn_transform(x, w, bias=b)
        assert torch.equal(y1, y0 + b)
    with pytest.raises(ValueError):
        gcn_transform(x, w, bias=b, dropout_p=1.0)
    with pytest.raises(ValueError):
        gcn_transform(x, w, bias=b, out_rows=torch.arange(x.shape[0], device=dev))
    for n in (1, 37, 20000, 300001):
        a = torch.randn(n, 128, device=dev, generator=gen)
        bb = torch.randn(n, 128, device=dev, generator=gen)
        c1, s1 = gemm_tn(a, bb, bb, trans=True)
        c2, s2 = gemm_tn(a, bb, bb.clone(), trans=True)
        assert torch.equal(c1, c2) and torch.equal(s1, s2)
        close(s1.cpu().numpy(), bb.double().sum(0).cpu().numpy(), rtol=1e-5)


@pytest.mark.parametrize("k,fo", [(128, 128), (64, 128), (256, 256)])
def test_transform_relu_dropout_epilogue(dev, k, fo):
    """gnn_gcn_transform_epi_f32: dropout_p(ReLU(x W^T + b)) equals the plain transform + b,
    ReLU and the oracle's hashed keep mask (oracle_dropout_keep over (row, column)) times
    1 / (1 - p), bit for bit at p = 0.5 (a power-of-two scale), to one rounding at p = 0.3;
    about 1 - p of the positive entries survive."""
    from graphneuralnetwork_amd.ops import gcn_transform
    gen = torch.Generator(device=dev).manual_seed(k + fo)
    n = 20011
    x = torch.randn(n, k, device=dev, generator=gen)
    w = torch.randn(fo, k, device=dev, generator=gen)
    b = torch.randn(fo, device=dev, generator=gen)
    base = torch.relu(gcn_transform(x, w) + b)
    for p, seed in ((0.5, 77), (0.3, 2 ** 61 + 5), (0.0, 0)):
        y = gcn_transform(x, w, relu=True, bias=b, dropout_p=p, seed=seed)
        keep = torch.from_numpy(c_oracle.dropout_keep(seed, np.arange(n)[:, None],
                                                      np.arange(fo)[None, :], p)).to(dev)
        ref = torch.where(keep, base * (1.0 / (1.0 - p)), torch.zeros((), device=dev))
        if p in (0.5, 0.0):
            assert torch.equal(y, ref)
        else:
            close(y.cpu().numpy(), ref.cpu().numpy(), rtol=1e-6)
        pos = base > 0
        frac = float((y[pos] > 0).float().mean())
        assert abs(frac - (1 - p)) < 0.01, frac
    y = gcn_transform(x, w, bias=b)  # bias only, no ReLU
    assert torch.equal(y, gcn_transform(x, w) + b)


@pytest.mark.parametrize("m,k", [(128, 128), (64, 128), (128, 64), (64, 64)])
@pytest.mark.parametrize("n", [1, 37, 20000, 300001])
def test_gemm_tn_masked(dev, m, k, n):
    """gnn_gemm_tn_masked_f32 (B' = B . [H > 0] * scale): equals gemm_tn over a B' formed in
    torch (with its column sums) bit for bit, and float64."""
    from graphneuralnetwork_amd.ops import gemm_tn, gemm_tn_masked
    gen = torch.Generator(device=dev).manual_seed(m + k + n)
    a = torch.randn(n, m, device=dev, generator=gen)
    b = torch.randn(n, k, device=dev, generator=gen)
    h = torch.relu(torch.randn(n, k, device=dev, generator=gen))
    bm = torch.where(h > 0, b * 2.0, torch.zeros((), device=dev))
    c, ds = gemm_tn_masked(a, b, h, 2.0, True, trans=True)
    c0, ds0 = gemm_tn(a, bm, bm, trans=True)
    assert torch.equal(c, c0) and torch.equal(ds, ds0)
    close(c.cpu().numpy(), (bm.double().t() @ a.double()).cpu().numpy(), rtol=1e-5)
    c1, none = gemm_tn_masked(a, b, h, 2.0, False)
    assert none is None and torch.equal(c1, c0.t())


@pytest.mark.parametrize("p", [0.0, 0.5])
@pytest.mark.parametrize("x_grad", [True, False])
def test_gcn_relu_dropout_fused_layer(dev, p, x_grad, monkeypatch):
    """Graph_conv_layer -> ReLU -> Dropout as one training op (ops.gcn_layer relu_dropout=):
    output and gradients (dW, db, and dX when X needs it) against the unfused layer followed by
    ReLU and the oracle's hashed keep mask times 1 / (1 - p) under torch autograd."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.gcn import Graph_conv_layer
    from graphneuralnetwork_amd.graph import CsrGraph
    rp, col, val = _rand_graph(3000, 30000, 6)
    g = CsrGraph(torch.from_numpy(rp).to(dev), torch.from_numpy(col).to(dev),
                 torch.from_numpy(val).to(dev), 3000, 3000)
    torch.manual_seed(1)
    layer = Graph_conv_layer(128, 128).to(dev)
    with torch.no_grad():
        layer.bias.normal_()
    X = torch.randn(3000, 128, device=dev)
    gy = torch.randn(3000, 128, device=dev)
    seed = 4242
    assert ops.fuses_relu_dropout(X, layer.dense.weight, g)
    xx = X.clone().requires_grad_(x_grad)
    h = ops.gcn_layer(g, xx, layer.dense.weight, layer.bias, relu_dropout=(p, seed))
    h.backward(gy)
    got = [h.detach(), layer.dense.weight.grad.clone(), layer.bias.grad.clone()] + (
        [xx.grad] if x_grad else [])
    layer.zero_grad(set_to_none=True)
    keep = torch.from_numpy(c_oracle.dropout_keep(seed, np.arange(3000)[:, None],
                                                  np.arange(128)[None, :], p)).to(dev)
    xr = X.clone().requires_grad_(x_grad)
    y = ops.gcn_layer(g, xr, layer.dense.weight, layer.bias)
    hr = torch.where(keep, torch.relu(y) * (1.0 / (1.0 - p)), torch.zeros((), device=dev))
    hr.backward(gy)
    ref = [hr.detach(), layer.dense.weight.grad, layer.bias.grad] + ([xr.grad] if x_grad else [])
    assert torch.equal(got[0], ref[0])
    for a, b in zip(got[1:], ref[1:]):
        close(a.cpu().numpy(), b.cpu().numpy())


def test_gcn_model_fused_training_equals_unfused(dev, monkeypatch):
    """GCN_Model(128, 128, 6, 3, 0).train(): the Graph_conv_layer -> ReLU -> Dropout triples run
    fused (gcn._fuse_train) and unfused (ops.GCN_FUSE_RELU_DROPOUT off) give the same logits and
    gradients to fp32 rounding; a forward hook on a ReLU turns the fusion off for its triple."""
    from graphneuralnetwork_amd import gcn as gcn_mod
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.gcn import GCN_Model
    from graphneuralnetwork_amd.graph import CsrGraph
    rp, col, val = _rand_graph(5000, 60000, 8)
    g = CsrGraph(torch.from_numpy(rp).to(dev), torch.from_numpy(col).to(dev),
                 torch.from_numpy(val).to(dev), 5000, 5000)
    torch.manual_seed(3)
    model = GCN_Model(128, 128, 6, 3, 0.0).to(dev).train()
    X = torch.randn(5000, 128, device=dev)
    lab = torch.randint(0, 6, (5000,), device=dev)
    spans = []
    real = gcn_mod._fuse_train
    monkeypatch.setattr(gcn_mod, "_fuse_train", lambda *a: spans.append(real(*a)) or spans[-1])
    res = {}
    for fuse in (True, False):
        monkeypatch.setattr(ops, "GCN_FUSE_RELU_DROPOUT", fuse)
        spans.clear()
        model.zero_grad(set_to_none=True)
        y = model(X, g)
        torch.nn.functional.cross_entropy(y, lab).backward()
        assert spans == ([3, 3, 0] if fuse else [0, 0, 0])
        res[fuse] = [y.detach()] + [p.grad.clone() for p in model.parameters()]
    for a, b in zip(res[True], res[False]):
        close(a.cpu().numpy(), b.cpu().numpy())
    monkeypatch.setattr(ops, "GCN_FUSE_RELU_DROPOUT", True)
    hk = model.gcn_blocks.relu0.register_forward_hook(lambda *a: None)
    spans.clear()
    model(X, g)
    hk.remove()
    assert spans[0] == 0 and spans[1] == 3


@pytest.mark.parametrize("k,fo", [(128, 8), (64, 7), (256, 16), (16, 1), (8, 128), (7, 64),
                                  (16, 256), (1, 128)])
@pytest.mark.parametrize("n", [1, 37, 20000, 300001])
def test_linear_small_vs_float64(dev, k, fo, n, monkeypatch):
    """gnn_linear_small_f32 (ops.linear_small, the classifier layer's support H W^T and its
    dX = dS W): x W^T against float64 with strided rows of x; uncovered shapes return None."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.ops import linear_small
    monkeypatch.setattr(ops, "LINEAR_SMALL_MAX_FOUT", 256)  # every shape the kernels take
    gen = torch.Generator(device=dev).manual_seed(k * 7 + fo + n)
    w = torch.randn(fo, k, device=dev, generator=gen)
    for x in (torch.randn(n, k + 4 + (-k) % 4, device=dev, generator=gen)[:, :k],
              torch.randn(n, k, device=dev, generator=gen)):  # an aligned pitch; rows of k
        y = linear_small(x, w)
        assert y is not None and y.shape == (n, fo)
        close(y.cpu().numpy(), (x.double() @ w.double().t()).cpu().numpy(), rtol=1e-5)
    assert linear_small(x, torch.randn(24, k, device=dev)) is None


def test_symmetric_graph_is_its_own_transpose(dev):
    """The GCN builders mark D^-1/2 (A_sym + I) D^-1/2 symmetric (no transposed copy); an
    unmarked graph whose transpose equals it (the reference's COO) is found to be so."""
    from graphneuralnetwork_amd.graph import CsrGraph, from_coo
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    s, d = rmat_edges(50_000, 400_000, 1)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), 50_000, device=dev)
    assert g.symmetric and g.transpose() is g
    rows = torch.repeat_interleave(torch.arange(g.n_rows, device=dev), g.rowptr[1:] - g.rowptr[:-1])
    t = from_coo(g.col.to(torch.int64), rows, g.val, g.n_cols, g.n_rows)
    assert torch.equal(t.rowptr, g.rowptr) and torch.equal(t.col, g.col)
    assert torch.allclose(t.val, g.val, rtol=2.0 ** -23, atol=0)
    plain = CsrGraph(g.rowptr, g.col, g.val, g.n_rows, g.n_cols)
    assert not plain.symmetric
    assert plain.transpose() is plain and plain.symmetric and plain._transpose is None


@pytest.mark.parametrize("order", ["natural", "degree"])
def test_gcn_layer_training_cfg2_full_size(dev, order):
    """The benchmarked training step at BASELINE cfg2 size (R-MAT 1M / 20.1M nnz, 128 -> 128)
    over the natural graph or the degree-ordered graph P A P^T GCN_Model trains over (degree:
    ops.gcn_train_order, XCD-direct hub plans in both directions), as (A X) W^T + b
    (ops.GCN_REASSOC): the forward equals the inference layer to fp32 rounding; the gradients
    equal float64
    references built from the C oracle's SpMM (dS = A dY, A symmetric) and numpy products
    (dX = dS W, dW = dS^T X, db = sum dY) on every row."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.gcn import Graph_conv_layer
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n = 1_000_000
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), n, device=dev)
    assert g.nnz == 20_073_500 and g.symmetric
    assert ops.column_order(g, 128) is not None
    if order == "degree":
        g = ops.gcn_train_order(g, 128).graph
        assert g.symmetric and ops.column_order(g, 128) is None
    gen = torch.Generator(device=dev).manual_seed(5)
    layer = Graph_conv_layer(128, 128).to(dev)
    with torch.no_grad():
        layer.bias.normal_(generator=gen)
    X = torch.randn(n, 128, device=dev, generator=gen)
    with torch.no_grad():
        y_inf = layer(X, g)
    y = layer(X, g)
    # training runs the 128 -> 128 layer as (A X) W^T + b (ops.GCN_REASSOC): the inference
    # layer's A (X W^T) + b regrouped
    close(y.detach().cpu().numpy(), y_inf.cpu().numpy())
    gy = torch.randn(n, 128, device=dev, generator=gen)
    y.backward(gy)
    assert g._transpose is None  # the symmetric graph served the backward itself
    rp, col, val = (t.cpu().numpy() for t in (g.rowptr, g.col, g.val))
    gyn = gy.cpu().numpy()
    dS = c_oracle.spmm_csr(rp, col, val, gyn).astype(np.float64)   # double accumulation
    Xn = X.cpu().numpy().astype(np.float64)
    W = layer.dense.weight.detach().cpu().numpy().astype(np.float64)
    close(layer.dense.weight.grad.cpu().numpy(), dS.T @ Xn)
    close(layer.bias.grad.cpu().numpy(), gyn.astype(np.float64).sum(0))
    X.requires_grad_(True)
    layer.zero_grad()
    layer(X, g).backward(gy)
    close(X.grad.cpu().numpy(), dS @ W)


def test_gcn_model_training_cfg2_full_size(dev, monkeypatch):
    """The whole benchmarked model's training step at cfg2 size: GCN_Model(128, 128, 7, 2, 0.5)
    (GCN/GCN.py:5-27, GCN/train_eval.py:43-48) as its forward runs it -- rows permuted onto
    P A P^T (PermuteRows); layer 1 128 -> 128 as (A X) W^T + b with ReLU and Dropout(0.5) in the
    transform's epilogue (one op: gcn._fuse_train), its dW / db on the masked gemm_tn; layer 2
    128 -> 7 (its weight gradient on the narrow gemm_tn kernel); logits permuted back. Each
    layer against float64 references (the C oracle's SpMM, numpy products, the oracle's hashed
    keep mask for the dropout seed the model drew) given the tensors the model handed it,
    captured in the permuted frame: layer 2's input and output by hooks on that layer, X's
    rows through the order's permutation. The ReLU mask is the model's own (H > 0), so no
    element near the kink can flip between fp32 and float64."""
    from graphneuralnetwork_amd import gcn as gcn_mod
    from graphneuralnetwork_amd.gcn import GCN_Model
    from graphneuralnetwork_amd.ops import gcn_train_order
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n, C, seed = 1_000_000, 7, 987654321
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), n, device=dev)
    del s, d
    torch.manual_seed(3)
    net = GCN_Model(128, 128, C, 2, 0.5).to(dev).train()
    gen = torch.Generator(device=dev).manual_seed(7)
    with torch.no_grad():
        for m in (net.gcn_blocks.gcn0, net.gcn_blocks.gcn1):
            m.bias.normal_(generator=gen)
    monkeypatch.setattr(gcn_mod, "dropout_seed", lambda: seed)
    spans = []
    real = gcn_mod._fuse_train
    monkeypatch.setattr(gcn_mod, "_fuse_train", lambda *a: spans.append(real(*a)) or spans[-1])
    seen = {}

    def keep(name):
        def hook(mod, inp, out=None):
            t = inp[0] if out is None else out
            t.retain_grad()
            seen[name] = t
        return hook

    net.gcn_blocks.gcn1.register_forward_pre_hook(keep("h"))
    net.gcn_blocks.gcn1.register_forward_hook(keep("y"))
    X = torch.randn(n, 128, device=dev, generator=gen).requires_grad_(True)
    gy = torch.randn(n, C, device=dev, generator=gen)
    Y = net(X, g)
    Y.backward(gy)
    assert spans == [3, 0]  # layer 1 + ReLU + Dropout fused; layer 2 alone
    order = gcn_train_order(g, 128)
    gp = order.graph
    perm = order.perm
    rp, col, val = (t.cpu().numpy() for t in (gp.rowptr, gp.col, gp.val))
    A = lambda v: c_oracle.spmm_csr(rp, col, val, v.astype(np.float32)).astype(np.float64)
    f64 = lambda t: t.detach().cpu().numpy().astype(np.float64)
    Xp, dXp = f64(X[perm]), f64(X.grad[perm])
    H, Hg, Yp, gyp = f64(seen["h"]), f64(seen["h"].grad), f64(seen["y"]), f64(seen["y"].grad)
    W1, b1 = f64(net.gcn_blocks.gcn0.dense.weight), f64(net.gcn_blocks.gcn0.bias)
    W2, b2 = f64(net.gcn_blocks.gcn1.dense.weight), f64(net.gcn_blocks.gcn1.bias)
    # layer 2 (128 -> 7) given the model's H and the logits' gradient
    close(Yp, A(H @ W2.T) + b2)
    dS2 = A(gyp)
    close(f64(net.gcn_blocks.gcn1.dense.weight.grad), dS2.T @ H)
    close(f64(net.gcn_blocks.gcn1.bias.grad), gyp.sum(0))
    close(Hg, dS2 @ W2)
    # layer 1 (128 -> 128, ReLU, Dropout 0.5 on the (seed, row, column) hash of the permuted
    # frame) given the model's input rows and the gradient layer 2 handed back
    kp = c_oracle.dropout_keep(seed, np.arange(n)[:, None], np.arange(128)[None, :], 0.5)
    assert abs(kp.mean() - 0.5) < 1e-3
    close(H, np.where(kp, np.maximum(A(Xp @ W1.T) + b1, 0.0) * 2.0, 0.0))
    dZ1 = Hg * (H > 0) * 2.0
    dS1 = A(dZ1)
    close(f64(net.gcn_blocks.gcn0.dense.weight.grad), dS1.T @ Xp)
    close(f64(net.gcn_blocks.gcn0.bias.grad), dZ1.sum(0))
    close(dXp, dS1 @ W1)


@pytest.mark.parametrize("m,k", [(128, 128), (64, 64), (128, 64), (64, 128), (8, 64),
                                 (16, 64), (128, 7), (64, 8), (128, 16), (2, 8), (2, 3), (1, 1),
                                 (33, 5)])
@pytest.mark.parametrize("n", [1, 37, 20000, 300001])
@pytest.mark.parametrize("prec", ["split-bf16", "fp32-mfma"])
def test_gemm_tn_vs_float64(dev, m, k, n, prec):
    """gnn_gemm_tn_f32 (the weight / bias gradients): A^T B and the column sums of D against
    float64, plain and transposed output, strided rows, an empty row range; deterministic. In
    both arithmetic modes (split-bf16: gemm_tn_x6_kernel, the default; fp32-mfma)."""
    from graphneuralnetwork_amd.ops import gemm_tn, set_transform_precision
    prev = set_transform_precision(prec)
    try:
        _gemm_tn_case(dev, m, k, n)
    finally:
        set_transform_precision(prev)


def _gemm_tn_case(dev, m, k, n):
    from graphneuralnetwork_amd.ops import gemm_tn
    gen = torch.Generator(device=dev).manual_seed(m + k + n)
    a = torch.randn(n, m + 4, device=dev, generator=gen)[:, :m]   # row stride m + 4
    b = torch.randn(n, k, device=dev, generator=gen)
    d = torch.randn(n, k, device=dev, generator=gen)
    c, ds = gemm_tn(a, b, d)
    ref = a.double().t() @ b.double()
    close(c.cpu().numpy(), ref.cpu().numpy(), rtol=1e-5)
    close(ds.cpu().numpy(), d.double().sum(0).cpu().numpy(), rtol=1e-5)
    ct, none = gemm_tn(a, b, trans=True)
    assert none is None and ct.shape == (k, m)
    assert torch.equal(ct, c.t())
    c2, ds2 = gemm_tn(a, b, d)
    assert torch.equal(c2, c) and torch.equal(ds2, ds)
    assert gemm_tn(torch.randn(n, 200, device=dev), b) is None  # uncovered: the caller's torch.mm


def test_gat_training_grads_use_tn_kernel(dev):
    """The GAT block's W / a gradients through _ProjectFn and _attention_vector_grads
    (gnn_gemm_tn_f32) equal float64 autograd of the same layer math."""
    from graphneuralnetwork_amd.gat import GAT
    from graphneuralnetwork_amd.graph import CsrGraph
    n = 3000
    rng = np.random.default_rng(9)
    r = np.concatenate([rng.integers(0, n, 30000), np.arange(n)])   # every row has an edge
    c = np.concatenate([rng.integers(0, n, 30000), np.arange(n)])
    order = np.lexsort((c, r))
    r, col = r[order], c[order].astype(np.int32)
    rowptr = np.zeros(n + 1, np.int64)
    np.add.at(rowptr, r + 1, 1)
    rowptr = np.cumsum(rowptr)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.ones(col.size, device=dev), n, n)
    net = GAT(64, 8, 3, dropout=0.0, alpha=0.2, nheads=8).to(dev).train()
    X = torch.randn(n, 64, device=dev)
    gy = torch.randn(n, 64, device=dev)
    net._heads(X, g).backward(gy)
    # float64 reference of the same block
    W = torch.cat([m.W for m in net.attentions], 1).detach().double().cpu().requires_grad_()
    a_s = torch.cat([m._a_parts()[0] for m in net.attentions]).detach().double().cpu()
    a_d = torch.cat([m._a_parts()[1] for m in net.attentions]).detach().double().cpu()
    a_s.requires_grad_()
    a_d.requires_grad_()
    Xd = X.double().cpu()
    rows = torch.from_numpy(np.repeat(np.arange(n), np.diff(rowptr)))
    cols = torch.from_numpy(col.astype(np.int64))
    Wh = (Xd @ W).view(n, 8, 8)
    el = (Wh * a_s.view(8, 8)).sum(-1)
    er = (Wh * a_d.view(8, 8)).sum(-1)
    z = torch.nn.functional.leaky_relu(el[rows] + er[cols], 0.2)
    mx = torch.full((n, 8), -torch.inf, dtype=torch.float64).index_reduce(0, rows, z, "amax")
    p = torch.exp(z - mx[rows])
    den = torch.zeros(n, 8, dtype=torch.float64).index_add(0, rows, p)
    num = torch.zeros(n, 8, 8, dtype=torch.float64).index_add(0, rows, p.unsqueeze(-1) * Wh[cols])
    out = torch.nn.functional.elu(num / den.unsqueeze(-1)).view(n, 64)
    out.backward(gy.double().cpu())
    gW = torch.cat([m.W.grad for m in net.attentions], 1).cpu().numpy()
    close(gW, W.grad.numpy())
    ga_s = torch.cat([m.a.grad.view(-1)[:8] for m in net.attentions]).cpu().numpy()
    ga_d = torch.cat([m.a.grad.view(-1)[8:] for m in net.attentions]).cpu().numpy()
    close(ga_s, a_s.grad.numpy())
    close(ga_d, a_d.grad.numpy())


@pytest.mark.parametrize("drop", [0.0, 0.5])
def test_gcn_model_first_layer_over_row_order(dev, monkeypatch, drop):
    """GCN_Model in training with input features that need no gradient: the first layer reads
    X in its original order through P A (ops.row_order_graph: rows relabelled, column ids as in
    A) instead of permuting X onto P A P^T -- logits and every parameter gradient equal the
    permuting path to fp32 rounding; P A is A's rows in the order's permutation, edges intact."""
    from graphneuralnetwork_amd import gcn as gcn_mod
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.gcn import GCN_Model
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    monkeypatch.setattr(ops, "XCD_MIN_NNZ", 0)
    monkeypatch.setattr(ops, "HUB_MIN_X_BYTES", 0)
    monkeypatch.setattr(gcn_mod, "dropout_seed", lambda: 12345)
    n = 60_000
    s, d = rmat_edges(n, 500_000, 5)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), n, device=dev)
    torch.manual_seed(0)
    model = GCN_Model(128, 128, 7, 2, drop).to(dev).train()
    X = torch.randn(n, 128, device=dev)
    lab = torch.randint(0, 7, (n,), device=dev)
    res, used = {}, {}
    for rows in (True, False):
        monkeypatch.setattr(ops, "GCN_FIRST_ROWS", rows)
        model.zero_grad(set_to_none=True)
        y = model(X, g)
        torch.nn.functional.cross_entropy(y, lab).backward()
        used[rows] = ("_nodeorder_rows",) in g._plans
        res[rows] = [y.detach()] + [p.grad.clone() for p in model.parameters()]
    assert used[True]
    for a, b in zip(res[True], res[False]):
        err = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        assert err < 1e-5, err
    o = ops.node_order(g)
    rg = ops.row_order_graph(g)
    deg = (g.rowptr[1:] - g.rowptr[:-1])[o.perm]
    assert torch.equal(rg.rowptr[1:] - rg.rowptr[:-1], deg)
    r = int(o.perm[7])
    a, b = int(rg.rowptr[7]), int(rg.rowptr[8])
    assert torch.equal(rg.col[a:b], g.col[int(g.rowptr[r]):int(g.rowptr[r + 1])])


def test_gcn_model_training_in_degree_order_equals_natural(dev, monkeypatch):
    """GCN_Model in training runs over P A P^T (ops.gcn_train_order: X permuted on entry, the
    logits on exit): logits and every gradient equal the natural-order step to fp32 rounding
    (dropout 0), X's gradient back in the original row order."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.gcn import GCN_Model
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    monkeypatch.setattr(ops, "XCD_MIN_NNZ", 0)
    monkeypatch.setattr(ops, "HUB_MIN_X_BYTES", 0)
    n = 60_000
    s, d = rmat_edges(n, 500_000, 3)
    torch.manual_seed(0)
    model = GCN_Model(128, 128, 6, 2, 0.0).to(dev).train()
    X = torch.randn(n, 128, device=dev)
    lab = torch.randint(0, 6, (n,), device=dev)
    res = {}
    for use in (True, False):
        monkeypatch.setattr(ops, "GCN_TRAIN_ORDER", use)
        g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), n, device=dev)
        xx = X.clone().requires_grad_(True)
        model.zero_grad(set_to_none=True)
        y = model(xx, g)
        torch.nn.functional.nll_loss(torch.nn.functional.log_softmax(y, 1), lab).backward()
        assert (("_nodeorder",) in g._plans) == use
        res[use] = [y.detach(), xx.grad] + [p.grad.clone() for p in model.parameters()]
    for a, b in zip(res[True], res[False]):
        err = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        assert err < 1e-5, err
