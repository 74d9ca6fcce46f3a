"""GCN aggregation (CSR SpMM) on the GPU vs the oracle and the reference's golden vectors.

Tolerance (north_star): fp32 within 1e-4 relative (atol scaled by max |y|);
integer/structure outputs bit-exact.
"""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from oracle import gnn_oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-4


def close(a, b, rtol=RTOL):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(1.0, float(np.nanmax(np.abs(b)))) if b.size else 1.0
    np.testing.assert_allclose(a, b, rtol=rtol, atol=1e-5 * scale)


def _graph(rowptr, col, val, n_cols, dev):
    from graphneuralnetwork_amd.graph import CsrGraph
    return CsrGraph(torch.as_tensor(rowptr, dtype=torch.int64, device=dev),
                    torch.as_tensor(col, dtype=torch.int32, device=dev),
                    torch.as_tensor(val, dtype=torch.float32, device=dev),
                    len(rowptr) - 1, n_cols)


def _ref_coo(g, name, dev):
    idx = np.stack([g[f"{name}_row"], g[f"{name}_col"]]).astype(np.int64)
    n = int(g[f"{name}_n"])
    return torch.sparse_coo_tensor(torch.from_numpy(idx), torch.from_numpy(g[f"{name}_val"]),
                                   (n, n)).to(dev)


def test_golden_spmm_layers(golden, dev):
    """Graph_conv_layer drop-in on the reference's own uncoalesced COO adjacency."""
    from graphneuralnetwork_amd.gcn import Graph_conv_layer
    g = golden("gcn_spmm")
    for name, feats in zip(g["cases"], g["feats"]):
        adj = _ref_coo(g, name, dev)
        for F in map(int, str(feats).split(",")):
            layer = Graph_conv_layer(F, F).to(dev)
            with torch.no_grad():
                layer.dense.weight.copy_(torch.eye(F))
                layer.bias.copy_(torch.from_numpy(g[f"{name}_F{F}_bias"]))
                X = torch.from_numpy(g[f"{name}_F{F}_xq"].astype(np.float32) / 8).to(dev)
                Y = layer(X, adj).cpu().numpy()
            rows = g[f"{name}_F{F}_rows"]
            close(Y[rows], g[f"{name}_F{F}_y"])


def test_golden_gcn_cora_model(golden, dev):
    """GCN_Model drop-in (reference state_dict keys) reproduces the reference logits."""
    from graphneuralnetwork_amd.gcn import GCN_Model
    g = golden("gcn_cora")
    n, nf = int(g["n"]), int(g["n_feat"])
    X = np.zeros((n, nf), np.float32)
    X[g["feat_row"], g["feat_col"].astype(np.int64)] = g["feat_val"]
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([g["adj_row"], g["adj_col"]]).astype(np.int64)),
                                  torch.from_numpy(g["adj_val"]), (n, n)).to(dev)
    model = GCN_Model(nf, num_hidden=128, num_classes=7, num_layers=2, dropout=0.5)
    sd = {"gcn_blocks.gcn0.dense.weight": g["w0"], "gcn_blocks.gcn0.bias": g["b0"],
          "gcn_blocks.gcn1.dense.weight": g["w1"], "gcn_blocks.gcn1.bias": g["b1"]}
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.to(dev).eval()
    with torch.no_grad():
        logits = model(torch.from_numpy(X).to(dev), adj).cpu().numpy()
    close(logits, g["logits"])


def _rand_graph(n, e, seed, hub_deg=0, n_cols=None):
    rng = np.random.default_rng(seed)
    n_cols = n if n_cols is None else n_cols
    src = rng.integers(0, n, e)
    dst = rng.integers(0, n_cols, e)
    if hub_deg:
        src = np.concatenate([src, np.full(hub_deg, 3), np.full(hub_deg // 2, n - 1)])
        dst = np.concatenate([dst, rng.integers(0, n_cols, hub_deg + hub_deg // 2)])
    val = rng.standard_normal(src.size).astype(np.float32)
    return O.coo_to_csr(src, dst, val, n)


@pytest.mark.parametrize("F", [1, 3, 7, 8, 16, 33, 64, 96, 128, 256, 300, 512, 1000, 2100])
def test_spmm_feature_widths(dev, F):
    from graphneuralnetwork_amd.ops import spmm_forward
    n = 700 if F < 1000 else 300
    rowptr, col, val = _rand_graph(n, 9 * n, F, hub_deg=700)
    rng = np.random.default_rng(F)
    X = rng.standard_normal((n, F)).astype(np.float32)
    b = rng.standard_normal(F).astype(np.float32)
    g = _graph(rowptr, col, val, n, dev)
    Y = spmm_forward(g, torch.from_numpy(X).to(dev), torch.from_numpy(b).to(dev)).cpu().numpy()
    close(Y, O.spmm_csr(rowptr, col, val, X, b))


@pytest.mark.parametrize("seg_len", [1, 2, 7, 64, 1000])
def test_long_row_split(dev, seg_len):
    """Rows above seg_len are cut into segments + fixed-order fix-up; every split agrees."""
    from graphneuralnetwork_amd.ops import spmm_forward
    n, F = 500, 128
    rowptr, col, val = _rand_graph(n, 20 * n, 11, hub_deg=3000)
    X = np.random.default_rng(1).standard_normal((n, F)).astype(np.float32)
    g = _graph(rowptr, col, val, n, dev)
    Y = spmm_forward(g, torch.from_numpy(X).to(dev), seg_len=seg_len).cpu().numpy()
    close(Y, O.spmm_csr(rowptr, col, val, X))
    plan = g.plan(seg_len)
    deg = np.diff(rowptr)
    assert plan.n_long == int((deg > seg_len).sum())
    assert plan.n_seg == int(np.ceil(deg[deg > seg_len] / seg_len).sum())
    np.testing.assert_array_equal(plan.long_row.cpu().numpy(), np.nonzero(deg > seg_len)[0])


def test_plan_fill_matches_host(dev):
    from graphneuralnetwork_amd.graph import CsrGraph
    rng = np.random.default_rng(3)
    deg = rng.zipf(1.6, size=20000).clip(0, 50000)
    deg[rng.random(deg.size) < 0.2] = 0
    rowptr = np.zeros(deg.size + 1, np.int64)
    np.cumsum(deg, out=rowptr[1:])
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.zeros(int(rowptr[-1]), dtype=torch.int32, device=dev),
                 torch.zeros(int(rowptr[-1]), device=dev), deg.size, 1)
    T = 37
    p = g.plan(T)
    seg_row, seg_begin = [], []
    for r in np.nonzero(deg > T)[0]:
        for e in range(0, deg[r], T):
            seg_row.append(r)
            seg_begin.append(rowptr[r] + e)
    np.testing.assert_array_equal(p.seg_row.cpu().numpy(), seg_row)
    np.testing.assert_array_equal(p.seg_begin.cpu().numpy(), seg_begin)
    ptr = p.long_seg_ptr.cpu().numpy()
    assert ptr[0] == 0 and ptr[-1] == len(seg_row)
    np.testing.assert_array_equal(np.diff(ptr), np.ceil(deg[deg > T] / T).astype(int))
    small = np.nonzero(deg <= 1)[0]
    np.testing.assert_array_equal(p.small_row.cpu().numpy(), small)
    np.testing.assert_array_equal(p.mid_row.cpu().numpy(), np.nonzero((deg > 1) & (deg <= T))[0])
    assert (p.small_col.cpu().numpy()[deg[small] == 0] == -1).all()
    assert p.n_small + p.n_mid + p.n_long == deg.size


def test_no_plan_path_matches(dev):
    """mid_row = NULL (the INTEGRATION.md stub): every row by one wave, same result."""
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.ops import spmm_forward
    n, F = 2000, 64
    rowptr, col, val = _rand_graph(n, 30 * n, 21, hub_deg=5000)
    g = _graph(rowptr, col, val, n, dev)
    X = torch.randn(n, F, device=dev)
    b = torch.randn(F, device=dev)
    y = torch.empty(n, F, device=dev)
    lib = _lib.load()
    rc = lib.gnn_spmm_csr_f32(g.rowptr.data_ptr(), g.col.data_ptr(), g.val.data_ptr(), n,
                              X.data_ptr(), F, F, b.data_ptr(), y.data_ptr(), F,
                              1, None, None, 0, None, None, 0, None, None, None, 0, None, 0,
                              None, 0, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    close(y.cpu().numpy(), spmm_forward(g, X, b).cpu().numpy())
    close(y.cpu().numpy(), O.spmm_csr(rowptr, col, val, X.cpu().numpy(), b.cpu().numpy()))


def test_empty_rows_edges_and_strides(dev):
    from graphneuralnetwork_amd.ops import spmm_forward
    n = 300
    rowptr, col, val = _rand_graph(n, 200, 5)  # mostly empty rows
    F = 64
    X = np.random.default_rng(0).standard_normal((n, 2 * F)).astype(np.float32)
    g = _graph(rowptr, col, val, n, dev)
    Xd = torch.from_numpy(X).to(dev)[:, 10:10 + F]  # row stride 128, 8-B misaligned start
    out = torch.full((n, F + 3), 7.0, device=dev)[:, :F]
    spmm_forward(g, Xd, out=out)
    close(out.cpu().numpy(), O.spmm_csr(rowptr, col, val, X[:, 10:10 + F]))
    # zero-edge graph
    g0 = _graph(np.zeros(n + 1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.float32), n, dev)
    b = torch.arange(F, dtype=torch.float32, device=dev)
    Y = spmm_forward(g0, torch.from_numpy(X[:, :F]).to(dev), b).cpu().numpy()
    np.testing.assert_array_equal(Y, np.broadcast_to(np.arange(F, dtype=np.float32), (n, F)))


def test_rectangular_and_activations(dev):
    from graphneuralnetwork_amd.ops import spmm_forward
    n, m, F = 400, 900, 128
    rowptr, col, val = _rand_graph(n, 5000, 2, n_cols=m)
    X = np.random.default_rng(2).standard_normal((m, F)).astype(np.float32)
    g = _graph(rowptr, col, val, m, dev)
    ref = O.spmm_csr(rowptr, col, val, X)
    Xd = torch.from_numpy(X).to(dev)
    close(spmm_forward(g, Xd, activation="relu").cpu().numpy(), np.maximum(ref, 0))
    close(spmm_forward(g, Xd, activation="elu").cpu().numpy(), np.where(ref > 0, ref, np.expm1(ref)))


def test_deterministic(dev):
    from graphneuralnetwork_amd.ops import spmm_forward
    n, F = 3000, 128
    rowptr, col, val = _rand_graph(n, 40 * n, 9, hub_deg=20000)
    X = torch.randn(n, F, device=dev)
    g = _graph(rowptr, col, val, n, dev)
    a = spmm_forward(g, X, seg_len=100)
    b = spmm_forward(g, X, seg_len=100)
    assert torch.equal(a, b)


def test_backward_matches_dense(dev):
    from graphneuralnetwork_amd.ops import spmm
    n, F = 200, 16
    rowptr, col, val = _rand_graph(n, 1500, 4)
    g = _graph(rowptr, col, val, n, dev)
    A = torch.zeros(n, n, dtype=torch.float64)
    for r in range(n):
        for e in range(rowptr[r], rowptr[r + 1]):
            A[r, col[e]] += float(val[e])
    X = torch.randn(n, F, device=dev, requires_grad=True)
    b = torch.randn(F, device=dev, requires_grad=True)
    Y = spmm(g, X, b)
    gy = torch.randn_like(Y)
    Y.backward(gy)
    close(X.grad.cpu().numpy(), (A.T @ gy.cpu().double()).numpy())
    close(b.grad.cpu().numpy(), gy.sum(0).cpu().numpy())


def test_rmat_1m_parity_vs_c_oracle(dev):
    """Full BASELINE cfg2 graph (RMAT 1M nodes, nnz 20,073,500): checked on a row sample + checksums."""
    from graphneuralnetwork_amd.ops import spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_normalized_csr
    from graphneuralnetwork_amd.rmat import rmat_edges
    n = 1_000_000
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_normalized_csr(s, d, n, device=dev)
    assert g.nnz == 20_073_500
    F = 128
    X = torch.randn(n, F, generator=torch.Generator().manual_seed(0)).to(dev)
    Yd = spmm_forward(g, X)  # X is 512 MB: the default path is the XCD-sliced hub staging
    assert any(isinstance(k, tuple) and k[0] == "_xcd" and v is not None
               for k, v in g._plans.items())
    assert torch.equal(Yd, spmm_forward(g, X))           # reproducible
    close(Yd.cpu().numpy(), spmm_forward(g, X, hubs=0).cpu().numpy(), rtol=1e-5)
    assert torch.equal(spmm_forward(g, X, hubs=131072), spmm_forward(g, X, hubs=0))
    Y = Yd.cpu().numpy()
    rowptr, col, val = g.rowptr.cpu().numpy(), g.col.cpu().numpy(), g.val.cpu().numpy()
    deg = np.diff(rowptr)
    rows = np.unique(np.concatenate([np.random.default_rng(0).choice(n, 4000, replace=False),
                                     np.argsort(-deg)[:64]]))
    Xn = X.cpu().numpy()
    ref = np.concatenate([c_oracle.spmm_csr(rowptr, col, val, Xn, None, r, r + 1) for r in rows])
    close(Y[rows], ref)
    # size-independent property: column sums of Y == (1^T A) X  (linearity)
    colsum_a = np.bincount(col, weights=val.astype(np.float64), minlength=n)
    np.testing.assert_allclose(Y.astype(np.float64).sum(0), colsum_a @ Xn.astype(np.float64),
                               rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("F", [3, 64, 128, 256, 600, 2100])
def test_hub_staging_bitexact(dev, F):
    """gnn_spmm_csr_hub_f32: staging the hottest rows of X into a compact table changes no
    bit of Y (same edge order; the gathered values are copies) for any hub count, with
    bias / activation / accumulate epilogues, long-row segments and strided X."""
    from graphneuralnetwork_amd.ops import spmm_forward
    n = 900
    rowptr, col, val = _rand_graph(n, 12 * n, 40 + F, hub_deg=4000)
    g = _graph(rowptr, col, val, n, dev)
    Xw = torch.randn(n, F + 5, device=dev)
    for X in (Xw[:, :F].contiguous(), Xw[:, 1:F + 1]):   # vector path and strided/misaligned
        b = torch.randn(F, device=dev)
        base = torch.randn(n, F, device=dev)
        for seg_len in (None, 16):
            ref = spmm_forward(g, X, b, activation="relu", seg_len=seg_len, hubs=0)
            acc_ref = spmm_forward(g, X, None, out=base.clone(), accumulate=True, seg_len=seg_len,
                                   hubs=0)
            for k in (1, 17, 300, n):
                y = spmm_forward(g, X, b, activation="relu", seg_len=seg_len, hubs=k)
                assert torch.equal(y, ref), (F, seg_len, k)
                y = spmm_forward(g, X, None, out=base.clone(), accumulate=True, seg_len=seg_len,
                                 hubs=k)
                assert torch.equal(y, acc_ref), (F, seg_len, k, "accumulate")
    close(ref.cpu().numpy(), np.maximum(O.spmm_csr(rowptr, col, val, X.cpu().numpy(),
                                                   b.cpu().numpy()), 0))


def _xcd_graph(n, seed):
    """Random rows with hubs, plus the corner rows of the XCD-sliced plan: one-edge rows
    whose edge is a hub column (rows 0-99), edgeless rows (100-109), and rows whose every
    edge is a duplicate of one hub column (110-119: a single partial ref left in pass 2)."""
    rng = np.random.default_rng(seed)
    src = rng.integers(120, n, 16 * n)
    dst = rng.integers(0, n, 16 * n)
    hub = np.concatenate([np.full(5000, 3), np.full(2500, n - 1)])
    src = np.concatenate([src, hub, np.arange(100), np.repeat(np.arange(110, 120), 8)])
    dst = np.concatenate([dst, rng.integers(0, n, hub.size), np.full(100, 7),
                          np.full(80, 11)])
    # columns 7 and 11 become the two hottest
    src = np.concatenate([src, rng.integers(120, n, 6000)])
    dst = np.concatenate([dst, np.repeat([7, 11], 3000)])
    val = rng.standard_normal(src.size).astype(np.float32)
    return O.coo_to_csr(src, dst, val, n)


@pytest.mark.parametrize("F", [3, 64, 128, 256, 600])
def test_xcd_hub_staging(dev, F, monkeypatch):
    """XCD-sliced hub staging (graph.XcdHubPlan, two hub-kernel passes over [table |
    partials]): equal to the unstaged kernel within fp32 rounding, bitwise reproducible,
    with bias / activation / accumulate epilogues, long-row segments and strided X."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.ops import spmm_forward
    monkeypatch.setattr(ops, "XCD_MIN_DEG", 4)     # many small items on a small graph
    monkeypatch.setattr(ops, "XCD_CHUNK", 8)
    n = 1500
    rowptr, col, val = _xcd_graph(n, 90 + F)
    g = _graph(rowptr, col, val, n, dev)
    Xw = torch.randn(n, F + 5, device=dev)
    for X in (Xw[:, :F].contiguous(), Xw[:, 1:F + 1]):
        b = torch.randn(F, device=dev)
        base = torch.randn(n, F, device=dev)
        for seg_len in (None, 16):
            ref = spmm_forward(g, X, b, activation="elu", seg_len=seg_len, hubs=0)
            acc_ref = spmm_forward(g, X, None, out=base.clone(), accumulate=True, seg_len=seg_len,
                                   hubs=0)
            for k, ph, ik in ((8, 1, None), (200, 1, None), (n, 1, None), (200, 2, None),
                              (n, 4, None), (n, 1, 64), (200, 2, 100)):
                monkeypatch.setattr(ops, "XCD_PHASES", ph)  # slices per XCD, in launch order
                monkeypatch.setattr(ops, "XCD_ITEM_ROWS", ik)  # items from the ik hottest rows
                y = spmm_forward(g, X, b, activation="elu", seg_len=seg_len, hubs=k, xcd=True)
                key = ("_xcd", k, 4, min(8, seg_len or 10 ** 9), ph, ik, None)
                assert g._plans.get(key) is not None, key
                close(y.cpu().numpy(), ref.cpu().numpy(), rtol=1e-5)
                assert torch.equal(y, spmm_forward(g, X, b, activation="elu", seg_len=seg_len,
                                                   hubs=k, xcd=True))
                y = spmm_forward(g, X, None, out=base.clone(), accumulate=True, seg_len=seg_len,
                                 hubs=k, xcd=True)
                close(y.cpu().numpy(), acc_ref.cpu().numpy(), rtol=1e-5)
    monkeypatch.setattr(ops, "XCD_PHASES", 1)
    monkeypatch.setattr(ops, "XCD_ITEM_ROWS", None)
    Xn = X.cpu().numpy()
    y = spmm_forward(g, X, b, hubs=n, xcd=True).cpu().numpy()
    close(y, O.spmm_csr(rowptr, col, val, Xn, b.cpu().numpy()))


def test_xcd_hub_default_policy(dev, monkeypatch):
    """The default: XCD slicing on graphs of >= XCD_MIN_NNZ entries whose X is staged; an
    explicit ``hubs`` keeps the bit-exact single-pass staging; no item -> single pass."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.ops import spmm_forward
    n, F = 2000, 128
    rowptr, col, val = _rand_graph(n, 30 * n, 5, hub_deg=6000)
    g = _graph(rowptr, col, val, n, dev)
    X = torch.randn(n, F, device=dev)
    monkeypatch.setattr(ops, "HUB_MIN_X_BYTES", 0)
    monkeypatch.setattr(ops, "XCD_MIN_NNZ", 1)
    y = spmm_forward(g, X)
    assert any(isinstance(k, tuple) and k[0] == "_xcd" for k in g._plans)
    close(y.cpu().numpy(), O.spmm_csr(rowptr, col, val, X.cpu().numpy()))
    g2 = _graph(rowptr, col, val, n, dev)
    assert torch.equal(spmm_forward(g2, X, hubs=64), spmm_forward(g2, X, hubs=0))
    assert not any(isinstance(k, tuple) and k[0] == "_xcd" for k in g2._plans)
    monkeypatch.setattr(ops, "XCD_MIN_DEG", 10 ** 9)   # no row qualifies: plan is None
    g3 = _graph(rowptr, col, val, n, dev)
    assert torch.equal(spmm_forward(g3, X), spmm_forward(g3, X, hubs=ops.hub_rows_for(n, F)))


def test_hub_plan_structure(dev):
    """col_hub decodes back to col; the hub set is the k highest column degrees."""
    n = 3000
    rowptr, col, val = _rand_graph(n, 20 * n, 77, hub_deg=9000)
    g = _graph(rowptr, col, val, n, dev)
    k = 123
    hp = g.hub_plan(k)
    ch = hp.col_hub.cpu().numpy().astype(np.int64)
    hub = hp.hub_ids.cpu().numpy()
    assert hp.k == k and len(np.unique(hub)) == k
    dec = np.where(ch < 0, hub[np.clip(-1 - ch, 0, k - 1)], ch)
    np.testing.assert_array_equal(dec, col)
    assert ((ch < 0) == np.isin(col, hub)).all()
    deg = np.bincount(col, minlength=n)
    assert deg[hub].min() >= np.delete(deg, hub).max()
    assert (np.diff(deg[hub]) <= 0).all()  # hottest first
    # deterministic: exactly the stable order (degree descending, ties by ascending id)
    np.testing.assert_array_equal(hub, np.lexsort((np.arange(n), -deg))[:k])
    assert int(hp.err.item()) == 0


@pytest.mark.parametrize("k,fout", [(16, 64), (32, 128), (64, 64), (64, 256), (128, 128),
                                    (256, 64), (256, 128), (128, 256), (256, 256)])
@pytest.mark.parametrize("n", [1, 63, 1000, 4097])
def test_gcn_transform_mfma(dev, k, fout, n):
    """gnn_gcn_transform_f32 (fp32 MFMA, W [fout, k] as nn.Linear) vs a float64 matmul;
    gnn_linear_relu_f32 = the same with max(., 0) (the SageLayer, GraphSAGE.py:18-20)."""
    from graphneuralnetwork_amd.ops import gcn_transform
    rng = np.random.default_rng(k * 7 + fout + n)
    X = rng.standard_normal((n, k + 4)).astype(np.float32)
    W = (rng.standard_normal((fout, k)) / np.sqrt(k)).astype(np.float32)
    ref = X[:, :k].astype(np.float64) @ W.astype(np.float64).T
    Xd = torch.from_numpy(X).to(dev)
    for x in (Xd[:, :k].contiguous(), Xd[:, :k]):   # packed and ldx = k + 4
        y = gcn_transform(x, torch.from_numpy(W).to(dev))
        assert y is not None and y.shape == (n, fout)
        close(y.cpu().numpy(), ref)
        yr = gcn_transform(x, torch.from_numpy(W).to(dev), relu=True)
        assert torch.equal(yr, torch.clamp_min(y, 0.0))


@pytest.mark.parametrize("k,fout", [(128, 64), (128, 128), (128, 256), (256, 64), (256, 128),
                                    (256, 256)])
@pytest.mark.parametrize("n", [37, 5000])
@pytest.mark.parametrize("scale", [1.0, 1e-3])
def test_transform_split_bf16_accuracy(dev, k, fout, n, scale):
    """The split-bf16 transform (fp32 products from bf16 MFMAs, gnn_transform_set_precision(1),
    the default at K >= 128) against a float64 product: its error, relative to sum_k |x w| of
    each output (the scale of a dot product's rounding), stays below 1e-6 and within 4x of the
    fp32-MFMA path's own error (mode 0, a k-ordered fp32 fmaf chain); every epilogue."""
    from graphneuralnetwork_amd.ops import (gcn_transform, linear_relu_classify,
                                            set_transform_precision)
    g = torch.Generator(device=dev).manual_seed(k + fout + n)
    x = torch.randn(n, k, device=dev, generator=g) * scale
    w = torch.randn(fout, k, device=dev, generator=g) / k ** 0.5
    xd, wd = x.double(), w.double()
    ref = xd @ wd.T
    mag = x.abs().double() @ w.abs().double().T
    errs = {}
    prev = set_transform_precision("split-bf16")
    try:
        for mode in ("fp32-mfma", "split-bf16"):
            set_transform_precision(mode)
            y = gcn_transform(x, w)
            assert y is not None
            errs[mode] = float(((y.double() - ref).abs() / mag.clamp_min(1e-300)).max())
            yr = gcn_transform(x, w, relu=True)
            assert torch.equal(yr, torch.clamp_min(y, 0.0))
            perm = torch.randperm(n, device=dev, generator=g)
            ys = gcn_transform(x, w, out=torch.empty_like(y), out_rows=perm)
            assert torch.equal(ys[perm], y)
            if fout <= 128:
                wcls = torch.randn(3, fout, device=dev, generator=g)
                y2, lg = linear_relu_classify(x, w, wcls, None)
                assert torch.equal(y2, yr)
                lref = yr.double() @ wcls.double().T
                close(lg.cpu().numpy(), lref.cpu().numpy(), rtol=1e-5)
    finally:
        set_transform_precision(prev)
    assert errs["split-bf16"] < 1e-6, errs
    assert errs["split-bf16"] <= 4 * errs["fp32-mfma"] + 1e-7, errs


def test_gcn_transform_fallback_and_training(dev):
    """Uncovered shapes return None (nn.Linear runs); with autograd the layer is ops.gcn_layer
    (its own backward, tests/test_training_gpu.py) and equals the inference path."""
    from graphneuralnetwork_amd.gcn import Graph_conv_layer
    from graphneuralnetwork_amd.ops import gcn_transform
    x = torch.randn(100, 7, device=dev)
    assert gcn_transform(x, torch.randn(5, 7, device=dev)) is None
    assert gcn_transform(torch.randn(100, 100, device=dev), torch.randn(128, 100, device=dev)) is None
    assert gcn_transform(torch.randn(100, 128, device=dev), torch.randn(96, 128, device=dev),
                         relu=True) is None
    n = 300
    rowptr, col, val = _rand_graph(n, 3000, 8)
    g = _graph(rowptr, col, val, n, dev)
    layer = Graph_conv_layer(128, 128).to(dev)
    X = torch.randn(n, 128, device=dev, requires_grad=True)
    y = layer(X, g)
    y.sum().backward()
    assert X.grad is not None and layer.dense.weight.grad is not None
    with torch.no_grad():
        y2 = layer(X, g)  # MFMA transform path
    close(y2.cpu().numpy(), y.detach().cpu().numpy())


@pytest.mark.parametrize("F", [36, 64, 128, 256, 512, 2100])
def test_packed_tasks_vs_oracle(dev, F, monkeypatch):
    """gnn_spmm_csr_tasks_f32 (short rows streamed a task of <= 63 rows per wave): against
    the C oracle for several task shapes, with runs of edgeless rows, long-row segments,
    hub staging, bias / activation, and accumulate with edgeless rows left unwritten; and
    against the one-wave-per-row kernel."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import CsrGraph
    rng = np.random.default_rng(F)
    n = 3000 if F < 1000 else 800
    deg = rng.integers(0, 12, n)
    deg[rng.integers(0, n, 30)] = rng.integers(60, 700, 30)
    deg[100:190] = 0                                   # a run longer than one task
    deg[500:503] = 0
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    col = rng.integers(0, n, rowptr[-1]).astype(np.int32)
    val = rng.standard_normal(rowptr[-1]).astype(np.float32)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.from_numpy(val).to(dev), n, n)
    X = rng.standard_normal((n, F)).astype(np.float32)
    b = rng.standard_normal(F).astype(np.float32)
    Xd, bd = torch.from_numpy(X).to(dev), torch.from_numpy(b).to(dev)
    ref = O.spmm_csr(rowptr, col, val, X, b)
    monkeypatch.setattr(ops, "SPMM_TASKS", False)
    per_row = ops.spmm_forward(g, Xd, bd, seg_len=256, hubs=0)
    monkeypatch.setattr(ops, "SPMM_TASKS", True)
    for max_deg, cost in ((1, 4), (8, 16), (64, 256), (128, 256), (700, 2048)):
        monkeypatch.setattr(ops, "TASK_MAX_DEG", max_deg)
        monkeypatch.setattr(ops, "TASK_COST", cost)
        for hubs in (0, 50):
            y = ops.spmm_forward(g, Xd, bd, seg_len=256, hubs=hubs)
            assert any(k[0] == "_tasks" for k in g._plans if isinstance(k, tuple))
            close(y.cpu().numpy(), ref)
            close(y.cpu().numpy(), per_row.cpu().numpy(), rtol=1e-5)
        y = ops.spmm_forward(g, Xd, bd, activation="elu", seg_len=256, hubs=0)
        close(y.cpu().numpy(), np.where(ref > 0, ref, np.expm1(np.minimum(ref, 0))))
        base = rng.standard_normal((n, F)).astype(np.float32)
        out = torch.from_numpy(base).to(dev)
        ops.spmm_forward(g, Xd, None, out=out, accumulate=True, seg_len=256, hubs=0)
        got = out.cpu().numpy()
        close(got, base + O.spmm_csr(rowptr, col, val, X))
        np.testing.assert_array_equal(got[deg == 0], base[deg == 0])  # never rewritten
    assert torch.equal(ops.spmm_forward(g, Xd, bd, seg_len=256),
                       ops.spmm_forward(g, Xd, bd, seg_len=256))  # deterministic


@pytest.mark.parametrize("F", [64, 128])
def test_packed_tasks_skip_empty_keeps_negative_zero(dev, F, monkeypatch):
    """ADVICE r3 (spmm.hip packed_rows): with GNN_EPI_SKIP_EMPTY an edgeless row inside a task
    is never written, so a -0.0 already in `out` keeps its sign bit (base + 0 would turn it into
    +0.0). Edgeless rows at every slot position of a task, after rows with edges (rp > 0)."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import CsrGraph
    rng = np.random.default_rng(F + 1)
    n = 4000
    deg = rng.integers(1, 6, n)
    deg[rng.random(n) < 0.4] = 0                       # edgeless rows scattered through tasks
    deg[700:760] = 0
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    col = rng.integers(0, n, rowptr[-1]).astype(np.int32)
    val = rng.standard_normal(rowptr[-1]).astype(np.float32)
    g = CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                 torch.from_numpy(val).to(dev), n, n)
    X = rng.standard_normal((n, F)).astype(np.float32)
    base = rng.standard_normal((n, F)).astype(np.float32)
    base[deg == 0] = -0.0
    for max_deg, cost in ((8, 16), (128, 256)):
        monkeypatch.setattr(ops, "TASK_MAX_DEG", max_deg)
        monkeypatch.setattr(ops, "TASK_COST", cost)
        out = torch.from_numpy(base).to(dev)
        ops.spmm_forward(g, torch.from_numpy(X).to(dev), None, out=out, accumulate=True,
                         seg_len=256, hubs=0)
        assert any(k[0] == "_tasks" for k in g._plans if isinstance(k, tuple))
        got = out.cpu().numpy()
        assert np.signbit(got[deg == 0]).all()
        close(got, base + O.spmm_csr(rowptr, col, val, X))


def test_packed_tasks_check(dev):
    """gnn_spmm_tasks_check flags tasks outside the contract (bit 1: empty, > 63 rows, out of
    range; bit 2: overlapping); the task kernel skips such tasks without reading past the
    graph; graph.check_tasks raises on them."""
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.graph import check_tasks
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    n = 200
    cases = (([0, 63, 63, 126], 0), ([0, 64], 1), ([5, 5], 1), ([190, 201], 1), ([-1, 3], 1),
             ([0, 10, 5, 20], 2))
    for tasks, want in cases:
        t = torch.tensor(tasks, dtype=torch.int32, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        assert lib.gnn_spmm_tasks_check(t.data_ptr(), t.numel() // 2, n, err.data_ptr(), s) == 0
        assert int(err.item()) == want, (tasks, int(err.item()))
        if want:
            with pytest.raises(ValueError):
                check_tasks(t, n)
    # the kernel itself: a 64-row task and an out-of-range one are skipped, the good one runs
    rowptr = torch.arange(n + 1, dtype=torch.int64, device=dev)
    col = torch.arange(n, dtype=torch.int32, device=dev)
    val = torch.ones(n, device=dev)
    F = 64
    X = torch.randn(n, F, device=dev)
    y = torch.full((n, F), 3.0, device=dev)
    bad = torch.tensor([0, 64, 100, 110, 150, 260], dtype=torch.int32, device=dev)
    mid = torch.zeros(1, dtype=torch.int32, device=dev)
    lsp = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = lib.gnn_spmm_csr_tasks_f32(rowptr.data_ptr(), col.data_ptr(), val.data_ptr(), n,
                                    X.data_ptr(), F, None, 0, F, None, y.data_ptr(), F, 256,
                                    None, None, 0, None, lsp.data_ptr(), 0, mid.data_ptr(), 0,
                                    bad.data_ptr(), 3, None, 0, s)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.equal(y[100:110], X[100:110])
    assert bool((y[:64] == 3.0).all()) and bool((y[150:] == 3.0).all())


def test_packed_tasks_c_abi_contract(dev):
    """gnn_spmm_csr_tasks_f32 rejects what it does not cover (feat not a multiple of 4,
    misaligned vectors) with GNN_E_UNSUPPORTED and unknown flags with GNN_E_ARG; narrow rows
    (feat 4 / 8 / 32: 1 / 2 / 8 lanes per row, 64 / 32 / 8 edge slots per wave) are
    covered."""
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.graph import CsrGraph
    lib = _lib.load()
    n = 64
    rowptr = torch.arange(n + 1, dtype=torch.int64, device=dev)
    col = torch.arange(n, dtype=torch.int32, device=dev)
    val = torch.ones(n, device=dev)
    g = CsrGraph(rowptr, col, val, n, n)
    tp = g.task_plan(256, 64, 128)
    s = torch.cuda.current_stream().cuda_stream
    for F, off, flags, want in ((6, 0, 0, _lib.E_UNSUPPORTED), (64, 1, 0, _lib.E_UNSUPPORTED),
                                (64, 0, 64, _lib.E_ARG), (64, 0, 0, 0), (32, 0, 0, 0),
                                (8, 0, 0, 0), (4, 0, 0, 0)):
        X = torch.randn(n, F + 4, device=dev)[:, off:off + F]
        y = torch.empty(n, F, device=dev)
        rc = lib.gnn_spmm_csr_tasks_f32(rowptr.data_ptr(), col.data_ptr(), val.data_ptr(), n,
                                        X.data_ptr(), X.stride(0), None, 0, F, None, y.data_ptr(),
                                        F, tp.seg_len, *tp.args(), None, flags, s)
        assert rc == want, (F, off, flags, rc)
        if rc == 0:
            torch.testing.assert_close(y, X)


@pytest.mark.parametrize("k", [128, 256])
def test_gcn_transform_wide_output_c_abi(dev, k):
    """gnn_gcn_transform_f32 at fout = 256 with k > 64 (one 8-wave x 2-block launch; the
    Python policy TRANSFORM_WIDE_MFMA routes Graph_conv_layer there): against a float64
    product."""
    from graphneuralnetwork_amd import _lib
    n = 3000
    x = torch.randn(n, k, device=dev)
    w = torch.randn(256, k, device=dev) / k ** 0.5
    y = torch.empty(n, 256, device=dev)
    lib = _lib.load()
    assert lib.gnn_gcn_transform_supported(k, 256)
    assert lib.gnn_gcn_transform_f32(x.data_ptr(), k, n, k, w.data_ptr(), 256, y.data_ptr(), 256,
                                     torch.cuda.current_stream().cuda_stream) == 0
    ref = (x.double() @ w.double().T).float()
    close(y.cpu().numpy(), ref.cpu().numpy())


@pytest.mark.parametrize("rows", [True, False])
@pytest.mark.parametrize("F", [64, 128, 600])
def test_xcd_direct_degree_order(dev, F, rows, monkeypatch):
    """On a degree-ordered graph (graph.degree_order) the XCD-sliced SpMM reads the hub rows
    in place (XcdHubPlan.prefix / direct: no staging copy). Its output is bit-identical to
    the staged copy's and to the natural-order graph's XCD result (the same items, slices
    and edge order), permuted; epilogues, accumulate, long-row segments."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import degree_order
    from graphneuralnetwork_amd.ops import spmm_forward
    monkeypatch.setattr(ops, "XCD_MIN_DEG", 4)
    monkeypatch.setattr(ops, "XCD_CHUNK", 8)
    n = 1500
    rowptr, col, val = _xcd_graph(n, 90 + F)
    g = _graph(rowptr, col, val, n, dev)
    o = degree_order(g, rows=rows)
    perm = o.perm
    X = torch.randn(n, F, device=dev)
    Xp = o.permute_rows(X)
    b = torch.randn(F, device=dev)
    base = torch.randn(n, F, device=dev)
    for seg_len in (None, 16):
        for k in (200, n):
            nat = spmm_forward(g, X, b, activation="relu", seg_len=seg_len, hubs=k, xcd=True)
            monkeypatch.setattr(ops, "XCD_DIRECT", True)
            y = spmm_forward(o.graph, Xp, b, activation="relu", seg_len=seg_len, hubs=k,
                             xcd=True)
            key = ("_xcd", k, 4, min(8, seg_len or 10 ** 9), 1, None, None)
            assert o.graph._plans[key].prefix
            monkeypatch.setattr(ops, "XCD_DIRECT", False)
            y_staged = spmm_forward(o.graph, Xp, b, activation="relu", seg_len=seg_len, hubs=k,
                                    xcd=True)
            assert torch.equal(y, y_staged)
            assert torch.equal(y, nat[perm] if rows else nat)
            monkeypatch.setattr(ops, "XCD_DIRECT", True)
            acc = spmm_forward(o.graph, Xp, None, out=(base[perm] if rows else base).clone(),
                               accumulate=True, seg_len=seg_len, hubs=k, xcd=True)
            acc_nat = spmm_forward(g, X, None, out=base.clone(), accumulate=True,
                                   seg_len=seg_len, hubs=k, xcd=True)
            assert torch.equal(acc, acc_nat[perm] if rows else acc_nat)
    y = spmm_forward(o.graph, Xp, b, hubs=n, xcd=True).cpu().numpy()
    want = O.spmm_csr(rowptr, col, val, X.cpu().numpy(), b.cpu().numpy())
    close(y, want[perm.cpu().numpy()] if rows else want)


@pytest.mark.parametrize("k,fout", [(64, 64), (128, 128), (256, 128), (64, 256), (256, 256)])
def test_transform_out_rows(dev, k, fout):
    """gnn_gcn_transform_rows_f32: y[out_rows[i]] = x[i] W^T, bit-identical to the in-order
    transform scattered (each row's MFMA chain does not depend on the others); a permutation,
    a scatter into a larger output (rows not named stay untouched), every tile size; an id out
    of range is not stored and raises."""
    from graphneuralnetwork_amd.ops import gcn_transform
    for n in (5000, 37, 1 << 17):
        x = torch.randn(n, k, device=dev)
        w = torch.randn(fout, k, device=dev) / k ** 0.5
        ref = gcn_transform(x, w)
        close(ref.cpu().numpy(), (x.double() @ w.double().T).cpu().numpy(), rtol=1e-5)
        perm = torch.randperm(n, device=dev)
        y = gcn_transform(x, w, out_rows=perm)
        want = torch.empty_like(ref)
        want[perm] = ref
        assert torch.equal(y, want)
        big = torch.full((2 * n + 3, fout), 7.0, device=dev)
        ids = torch.randperm(2 * n + 3, device=dev)[:n]
        gcn_transform(x, w, out=big, out_rows=ids)
        assert torch.equal(big[ids], ref)
        rest = torch.ones(2 * n + 3, dtype=torch.bool, device=dev)
        rest[ids] = False
        assert bool((big[rest] == 7.0).all())
    x = torch.randn(3, k, device=dev)
    w = torch.randn(fout, k, device=dev)
    bad = torch.tensor([0, 3, 1], device=dev)
    with pytest.raises(IndexError):
        gcn_transform(x, w, out_rows=bad)
    out = torch.zeros(3, fout, device=dev)
    gcn_transform(x, w, out=out, out_rows=bad, check_rows=False)
    assert torch.equal(out[2], torch.zeros(fout, device=dev))
    with pytest.raises(TypeError):
        gcn_transform(x, w, out_rows=bad.to(torch.int32))


def test_gcn_layer_column_order(dev, monkeypatch):
    """Graph_conv_layer on a graph that takes the XCD path: the inference forward runs over
    the column-degree-ordered graph (transform rows = perm, hub rows read in place) and
    returns the rows in the original order, bit-identical to the natural-order layer."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.gcn import Graph_conv_layer
    monkeypatch.setattr(ops, "HUB_MIN_X_BYTES", 0)
    monkeypatch.setattr(ops, "XCD_MIN_NNZ", 1)
    monkeypatch.setattr(ops, "XCD_MIN_DEG", 4)
    n, F = 2000, 128
    rowptr, col, val = _rand_graph(n, 30 * n, 5, hub_deg=6000)
    g = _graph(rowptr, col, val, n, dev)
    layer = Graph_conv_layer(64, F).to(dev)
    with torch.no_grad():
        layer.bias.normal_()
    X = torch.randn(n, 64, device=dev)
    with torch.no_grad():
        y = layer(X, g)
        assert ("_colorder",) in g._plans
        xp = next(p for key, p in g._plans[("_colorder",)].graph._plans.items()
                  if isinstance(key, tuple) and key[0] == "_xcd")
        assert xp is not None and xp.prefix
        monkeypatch.setattr(ops, "DEGREE_ORDER", False)
        y_nat = layer(X, _graph(rowptr, col, val, n, dev))
    assert torch.equal(y, y_nat)
    support = (X.double() @ layer.dense.weight.detach().double().T).cpu().numpy()
    close(y.cpu().numpy(), O.spmm_csr(rowptr, col, val, support, layer.bias.detach().cpu().numpy()),
          rtol=1e-4)


def test_in_degree_matches_bincount(dev):
    """gnn_in_degree_u32 (LDS-privatised counts for the hot ids, the hub plan's histogram) ==
    torch.bincount, on a power-law graph whose hubs are the smallest ids (degree-ordered) and
    on its natural order, incl. columns past the LDS range and columns without edges."""
    from graphneuralnetwork_amd.graph import CsrGraph, degree_order, in_degree
    rowptr, col, val = _rand_graph(50000, 900000, 3, hub_deg=40000)
    g = _graph(rowptr, col, val, 50000, dev)
    for gg in (g, degree_order(g, rows=False).graph):
        want = torch.bincount(gg.col.to(torch.int64), minlength=gg.n_cols)
        assert torch.equal(in_degree(gg), want)
    empty = CsrGraph(torch.zeros(3, dtype=torch.int64, device=dev),
                     torch.zeros(0, dtype=torch.int32, device=dev), torch.zeros(0, device=dev), 2, 9)
    assert torch.equal(in_degree(empty), torch.zeros(9, dtype=torch.int64, device=dev))


def test_gcn_model_relu_epilogue_equals_separate_relu(dev):
    """GCN_Model at inference runs each Graph_conv_layer + nn.ReLU pair (GCN/GCN.py:12-13) as
    one layer with the ReLU in the SpMM's store epilogue: equal to the layer followed by
    torch.relu, NaN included (torch.relu keeps NaN), on the column-ordered path of an R-MAT
    graph; a hook on the ReLU keeps the pair separate."""
    from graphneuralnetwork_amd.gcn import GCN_Model
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n = 300_000
    s, d = rmat_edges(n, 3_000_000, 2)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), n, device=dev)
    torch.manual_seed(4)
    model = GCN_Model(64, 128, 16, 3, 0.5).to(dev).eval()
    X = torch.randn(n, 64, device=dev)
    X[5, 3] = float("nan")
    with torch.no_grad():
        y = model(X, g)
        ref = X
        for b in model.gcn_blocks:
            ref = b(ref, g) if b._get_name() == "Graph_conv_layer" else b(ref)
        seen = []
        h = model.gcn_blocks.relu0.register_forward_hook(lambda *a: seen.append(1))
        y2 = model(X, g)
        h.remove()
    assert torch.isnan(y).any() and seen == [1]
    assert torch.equal(torch.nan_to_num(y, nan=7.0), torch.nan_to_num(ref, nan=7.0))
    assert torch.equal(torch.nan_to_num(y2, nan=7.0), torch.nan_to_num(ref, nan=7.0))


def test_spmm_replay_restores_the_plan(dev):
    """bench.spmm_replay (the measured SpMM ceiling: the product kernels with their gathered
    ids rewritten in place) leaves the plan as it found it: the step after the replay equals
    the step before it bit for bit, and the variants are timed in the expected order."""
    import bench
    from graphneuralnetwork_amd.ops import column_order, spmm_forward
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    n = 1_000_000
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s), torch.from_numpy(d), n, device=dev)
    ga = column_order(g, 128).graph
    X = torch.randn(n, 128, device=dev)
    b = torch.randn(128, device=dev)
    Y0 = spmm_forward(ga, X, b)
    Y = torch.empty_like(Y0)
    r = bench.spmm_replay(ga, X, b, Y, reps=2)
    assert r is not None and r["hub_rows"] > 0 and r["pass1_hub_gathers"] > 0
    assert r["all_gathers_in_L2_ms"] < r["as_built_ms"]
    assert torch.equal(spmm_forward(ga, X, b), Y0)
