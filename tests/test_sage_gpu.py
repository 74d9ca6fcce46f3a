"""GraphSAGE aggregation on the GPU vs the reference's golden vectors and the oracle.

MEAN: fp32 within 1e-4 relative; MAX (torch.argmax int64 indices): bit-exact."""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from oracle import gnn_oracle as O

pytestmark = pytest.mark.gpu


def close(a, b, rtol=1e-4):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(1.0, float(np.nanmax(np.abs(b)))) if b.size else 1.0
    np.testing.assert_allclose(a, b, rtol=rtol, atol=1e-5 * scale)


def _sd(g, tag):
    p = f"{tag}_sd_"
    return {k[len(p):]: torch.from_numpy(v) for k, v in g.items() if k.startswith(p)}


@pytest.mark.parametrize("tag,agg,gcn", [("mean", "MEAN", False), ("max", "MAX", False),
                                         ("gcn", "MEAN", True)])
def test_golden_graphsage_supervised(golden, dev, tag, agg, gcn):
    from graphneuralnetwork_amd.graphsage import Aggregator, GraphSAGE
    g = golden("sage")
    F = g["feat"].shape[1]
    net = GraphSAGE(2, F, 16, gcn, agg_func=agg, Unsupervised=False, class_size=3)
    net.load_state_dict(_sd(g, tag), strict=True)
    net.to(dev).eval()
    X = [torch.from_numpy(g[f"{tag}_{k}"]).to(dev)
         for k in ("center_feats", "nodes_map", "neigh_feats", "neigh_map")]
    with torch.no_grad():
        agg0 = Aggregator(X[2], agg).cpu().numpy()
        emb, logits = net(*X, None, None, None, None, None)
    if agg == "MAX":
        assert agg0.dtype == np.int64
        np.testing.assert_array_equal(agg0, g[f"{tag}_agg0"])
    else:
        close(agg0, g[f"{tag}_agg0"])
    close(emb.cpu().numpy(), g[f"{tag}_emb"])
    close(logits.cpu().numpy(), g[f"{tag}_logits"])


def test_golden_graphsage_unsupervised(golden, dev):
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    g = golden("sage")
    F = g["feat"].shape[1]
    net = GraphSAGE(2, F, 16, False, agg_func="MEAN", Unsupervised=True)
    net.load_state_dict(_sd(g, "unsup"), strict=True)
    net.to(dev).eval()
    X = [torch.from_numpy(g[f"unsup_X{i}"]).to(dev) for i in range(8)]
    with torch.no_grad():
        emb, scores = net(*X, tuple(int(v) for v in g["unsup_shape"]))
    close(emb.cpu().numpy(), g["unsup_emb"])
    close(scores.cpu().numpy(), g["unsup_scores"])


@pytest.mark.parametrize("F", [1, 7, 32, 100, 128, 256, 600, 2050])
@pytest.mark.parametrize("k", [1, 3, 10, 25, 70])
def test_pregathered_mean_and_argmax(dev, F, k):
    from graphneuralnetwork_amd.ops import sage_aggregate
    rng = np.random.default_rng(F * 100 + k)
    M = 300 if F < 1000 else 40
    x = (rng.integers(-6, 7, size=(M, k, F)) / 4).astype(np.float32)  # many ties
    x[0, min(1, k - 1), 0] = np.nan
    if k > 2:
        x[1, 2, : min(F, 3)] = np.nan
        x[1, k - 1, : min(F, 3)] = np.nan
    xd = torch.from_numpy(x).to(dev)
    close(sage_aggregate(xd, "MEAN").cpu().numpy()[2:], O.aggregator(x, "MEAN")[2:])
    got = sage_aggregate(xd, "MAX").cpu().numpy()
    np.testing.assert_array_equal(got, O.aggregator(x, "MAX"))
    np.testing.assert_array_equal(got, torch.argmax(torch.from_numpy(x), dim=1).numpy())


@pytest.mark.parametrize("F", [16, 128, 300])
def test_fused_gather_aggregate(dev, F):
    from graphneuralnetwork_amd.ops import gather_rows, sage_gather_aggregate
    rng = np.random.default_rng(F)
    n, M, k = 5000, 2000, 10
    table = (rng.integers(-8, 9, size=(n, F)) / 8).astype(np.float32)
    idx = rng.integers(0, n, size=(M, k))
    td = torch.from_numpy(table).to(dev)
    idd = torch.from_numpy(idx).to(dev)
    close(sage_gather_aggregate(td, idd, "MEAN").cpu().numpy(), O.sage_gather_aggregate(table, idx, "MEAN"))
    np.testing.assert_array_equal(sage_gather_aggregate(td, idd, "MAX").cpu().numpy(),
                                  O.sage_gather_aggregate(table, idx, "MAX"))
    np.testing.assert_array_equal(gather_rows(td, idd[:, 0]).cpu().numpy(), table[idx[:, 0]])


def test_out_of_range_indices_raise(dev):
    from graphneuralnetwork_amd.ops import gather_rows, sage_gather_aggregate
    t = torch.zeros(10, 8, device=dev)
    with pytest.raises(IndexError):
        sage_gather_aggregate(t, torch.tensor([[1, 10]], device=dev))
    with pytest.raises(IndexError):
        gather_rows(t, torch.tensor([-1], device=dev))


def test_mean_backward(dev):
    from graphneuralnetwork_amd.graphsage import Aggregator
    x = torch.randn(5, 4, 3, device=dev, requires_grad=True)
    y = Aggregator(x, "MEAN")
    y.backward(torch.ones_like(y))
    assert torch.allclose(x.grad, torch.full_like(x, 0.25))


@pytest.mark.parametrize("M,k,n,F", [(300, 10, 500, 64), (1000, 25, 120, 128), (7, 3, 5, 12)])
def test_gather_backward_is_the_transposed_aggregation(dev, M, k, n, F):
    """d table of the fused gather-mean / row gather (HIP SpMM over the transposed
    index map) vs torch autograd of table[idx].mean(1) / table[idx] in float64."""
    from graphneuralnetwork_amd.graphsage import Aggregator, Gathered, _gather
    gen = torch.Generator().manual_seed(M + k)
    table = torch.randn(n, F, generator=gen)
    idx = torch.randint(0, n, (M, k), generator=gen)
    ctr = torch.randint(0, n, (M,), generator=gen)
    gy = torch.randn(M, F, generator=gen)
    gz = torch.randn(M, F, generator=gen)
    t = table.to(dev).requires_grad_(True)
    y = Aggregator(Gathered(t, idx.to(dev)), "MEAN")
    z = _gather(t, ctr.to(dev))
    (y * gy.to(dev)).sum().add((z * gz.to(dev)).sum()).backward()
    t64 = table.double().requires_grad_(True)
    (t64[idx].mean(1) * gy.double()).sum().add((t64[ctr] * gz.double()).sum()).backward()
    ref = t64.grad.numpy()
    got = t.grad.cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=2e-5 * np.abs(ref).max())


@pytest.mark.parametrize("F,H", [(128, 128), (64, 128), (128, 256), (64, 256)])
@pytest.mark.parametrize("M,k", [(1, 1), (31, 3), (33, 10), (1000, 25), (4100, 10)])
def test_fused_sage_layer_vs_oracle(dev, F, H, M, k, monkeypatch):
    """gnn_sage_layer_f32: relu(W . cat[self, mean of k table rows]) in one launch (gathers
    into an LDS tile, v_mfma_f32_16x16x4_f32), with and without a centre index."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.ops import sage_layer
    monkeypatch.setattr(ops, "SAGE_FUSED_MIN_ROWS", 1)
    rng = np.random.default_rng(F + H + M + k)
    n = 5000
    table = rng.standard_normal((n, F)).astype(np.float32)
    idx = rng.integers(0, n, (M, k))
    cidx = rng.integers(0, n, M)
    W = (rng.standard_normal((H, 2 * F)) * 0.1).astype(np.float32)
    T, Wd = torch.from_numpy(table).to(dev), torch.from_numpy(W).to(dev)
    agg = table[idx].astype(np.float64).mean(1)
    for self_idx in (cidx, None):
        selfm = table[self_idx] if self_idx is not None else table[:M]
        ref = np.maximum(np.concatenate([selfm, agg], 1) @ W.T.astype(np.float64), 0)
        out = sage_layer(T, torch.from_numpy(idx).to(dev), Wd,
                         T if self_idx is not None else T[:M],
                         None if self_idx is None else torch.from_numpy(self_idx).to(dev))
        assert out is not None and out.shape == (M, H)
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-4,
                                   atol=1e-5 * max(1.0, np.abs(ref).max()))


def test_fused_sage_layer_checks_and_fallbacks(dev, monkeypatch):
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.ops import sage_layer
    monkeypatch.setattr(ops, "SAGE_FUSED_MIN_ROWS", 1)
    T = torch.randn(100, 128, device=dev)
    W = torch.randn(128, 256, device=dev)
    idx = torch.randint(0, 100, (10, 4), device=dev)
    bad = idx.clone()
    bad[3, 2] = 100
    with pytest.raises(IndexError):
        sage_layer(T, bad, W, T, torch.arange(10, device=dev))
    with pytest.raises(IndexError):
        sage_layer(T, idx, W, T, torch.full((10,), -1, device=dev))
    assert sage_layer(T, idx, torch.randn(96, 256, device=dev), T[:10]) is None   # H = 96
    assert sage_layer(T[:, :100], idx, torch.randn(128, 200, device=dev), T[:10, :100]) is None
    assert sage_layer(T, idx[:, :0], W, T[:10]) is None                            # k = 0


def test_graphsage_forward_fused_matches_unfused(dev, monkeypatch):
    """The eval-mode forward on device-sampler maps (Gathered inputs) gives the same
    embeddings and logits through the fused layer kernel as through gather-mean + GEMM."""
    from graphneuralnetwork_amd import graphsage as GS
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import from_coo
    from graphneuralnetwork_amd.sampler import sample_batch
    monkeypatch.setattr(ops, "SAGE_FUSED_MIN_ROWS", 1)
    rng = np.random.default_rng(7)
    n, F = 3000, 128
    s, d = rng.integers(0, n, 40000), rng.integers(0, n, 40000)
    adj = from_coo(torch.from_numpy(np.concatenate([s, d])).to(dev),
                   torch.from_numpy(np.concatenate([d, s])).to(dev),
                   torch.ones(80000, device=dev), n, n)
    table = torch.randn(n, F, device=dev)
    deg = adj.rowptr[1:] - adj.rowptr[:-1]
    seeds = torch.nonzero(deg > 0).view(-1)[:500]
    batch = sample_batch(adj, seeds, (25, 10), seed=3)
    net = GS.GraphSAGE(2, F, F, False, agg_func="MEAN", Unsupervised=False,
                       class_size=3).to(dev).eval()
    with torch.no_grad():
        emb, logits = net(*batch.forward_args(table), None, None, None, None, None)
        monkeypatch.setattr(GS, "sage_layer", lambda *a, **kw: None)
        emb0, logits0 = net(*batch.forward_args(table), None, None, None, None, None)
    np.testing.assert_allclose(emb.cpu().numpy(), emb0.cpu().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(logits.cpu().numpy(), logits0.cpu().numpy(), rtol=1e-4, atol=1e-5)


def test_graphsage_forward_mfma_gemm_matches_library(dev, monkeypatch):
    """The inference SageLayer GEMM relu([self | agg] @ W^T) on the hand-written fp32-MFMA
    kernel (gnn_linear_relu_f32, forced for every layer here) gives the embeddings and logits
    of the hipBLASLt GEMM within fp32 tolerance."""
    from graphneuralnetwork_amd import graphsage as GS
    from graphneuralnetwork_amd.graph import from_coo
    from graphneuralnetwork_amd.sampler import sample_batch
    rng = np.random.default_rng(11)
    n, F = 5000, 128
    s, d = rng.integers(0, n, 60000), rng.integers(0, n, 60000)
    adj = from_coo(torch.from_numpy(np.concatenate([s, d])).to(dev),
                   torch.from_numpy(np.concatenate([d, s])).to(dev),
                   torch.ones(120000, device=dev), n, n)
    table = torch.randn(n, F, device=dev)
    deg = adj.rowptr[1:] - adj.rowptr[:-1]
    seeds = torch.nonzero(deg > 0).view(-1)[:700]
    batch = sample_batch(adj, seeds, (25, 10), seed=5)
    net = GS.GraphSAGE(2, F, F, False, agg_func="MEAN", Unsupervised=False,
                       class_size=3).to(dev).eval()
    with torch.no_grad():
        monkeypatch.setattr(GS, "_sage_gemm_on_mfma", lambda rows: True)
        emb, logits = net(*batch.forward_args(table), None, None, None, None, None)
        monkeypatch.setattr(GS, "_sage_gemm_on_mfma", lambda rows: False)
        emb0, logits0 = net(*batch.forward_args(table), None, None, None, None, None)
    assert (emb >= 0).all()
    np.testing.assert_allclose(emb.cpu().numpy(), emb0.cpu().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(logits.cpu().numpy(), logits0.cpu().numpy(), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("k,fout", [(256, 128), (128, 128), (64, 64), (128, 256), (32, 128)])
@pytest.mark.parametrize("n", [1, 100, 8192, 20001])
@pytest.mark.parametrize("n_cls,bias", [(3, True), (1, False), (4, True)])
def test_linear_relu_classify(dev, k, fout, n, n_cls, bias):
    """gnn_linear_relu_cls_f32 (the last SageLayer with the classifier in its epilogue,
    GraphSAGE.py:18-20 + :51-52): the embedding equals gnn_linear_relu_f32 bit for bit and the
    logits equal a float64 (relu(x W^T)) wd^T + bd within fp32 tolerance; deterministic."""
    from graphneuralnetwork_amd.ops import gcn_transform, linear_relu_classify
    g = torch.Generator(device=dev).manual_seed(n * 7 + k + n_cls)
    x = torch.randn(n, k, device=dev, generator=g)
    w = torch.randn(fout, k, device=dev, generator=g) / k ** 0.5
    wd = torch.randn(n_cls, fout, device=dev, generator=g) / fout ** 0.5
    bd = torch.randn(n_cls, device=dev, generator=g) if bias else None
    if fout > 128:  # the epilogue covers up to 8 waves x 16 columns; nn.Linear runs instead
        assert linear_relu_classify(x, w, wd, bd) is None
        return
    y, lg = linear_relu_classify(x, w, wd, bd)
    assert torch.equal(y, gcn_transform(x, w, relu=True))
    ref = y.double() @ wd.double().T + (bd.double() if bias else 0.0)
    np.testing.assert_allclose(lg.cpu().numpy(), ref.cpu().numpy(), rtol=1e-5, atol=1e-5)
    y2, lg2 = linear_relu_classify(x, w, wd, bd)
    assert torch.equal(lg, lg2) and torch.equal(y, y2)


def test_linear_relu_classify_uncovered(dev):
    """More than 4 classes or an uncovered transform shape: None (the caller runs nn.Linear)."""
    from graphneuralnetwork_amd.ops import linear_relu_classify
    x = torch.randn(50, 128, device=dev)
    w = torch.randn(128, 128, device=dev)
    assert linear_relu_classify(x, w, torch.randn(5, 128, device=dev)) is None
    assert linear_relu_classify(torch.randn(50, 100, device=dev), torch.randn(128, 100, device=dev),
                                torch.randn(3, 128, device=dev)) is None
    with pytest.raises(ValueError):  # a caller-supplied out of the wrong shape
        linear_relu_classify(x, w, torch.randn(3, 128, device=dev),
                             out=torch.empty(49, 128, device=dev))


def test_graphsage_forward_classifier_epilogue(dev, monkeypatch):
    """The supervised forward on device-sampler maps with the classifier fused into the last
    SageLayer's GEMM gives the logits of the separate self.dense (nn.Linear) call."""
    from graphneuralnetwork_amd import graphsage as GS
    from graphneuralnetwork_amd.graph import from_coo
    from graphneuralnetwork_amd.sampler import sample_batch
    rng = np.random.default_rng(13)
    n, F = 4000, 128
    s, d = rng.integers(0, n, 50000), rng.integers(0, n, 50000)
    adj = from_coo(torch.from_numpy(np.concatenate([s, d])).to(dev),
                   torch.from_numpy(np.concatenate([d, s])).to(dev),
                   torch.ones(100000, device=dev), n, n)
    table = torch.randn(n, F, device=dev)
    deg = adj.rowptr[1:] - adj.rowptr[:-1]
    seeds = torch.nonzero(deg > 0).view(-1)[:600]
    batch = sample_batch(adj, seeds, (25, 10), seed=9)
    net = GS.GraphSAGE(2, F, F, False, agg_func="MEAN", Unsupervised=False,
                       class_size=3).to(dev).eval()
    calls = []
    real = GS.linear_relu_classify
    monkeypatch.setattr(GS, "linear_relu_classify",
                        lambda *a, **kw: calls.append(1) or real(*a, **kw))
    with torch.no_grad():
        emb, logits = net(*batch.forward_args(table), None, None, None, None, None)
        assert calls, "the classifier epilogue did not run"
        ref = net.dense(emb)
        monkeypatch.setattr(GS, "linear_relu_classify", lambda *a, **kw: None)
        emb0, logits0 = net(*batch.forward_args(table), None, None, None, None, None)
    assert torch.equal(emb, emb0)
    np.testing.assert_allclose(logits.cpu().numpy(), ref.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(logits.cpu().numpy(), logits0.cpu().numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("F", [1, 7, 128, 600])
@pytest.mark.parametrize("k", [1, 10, 25])
def test_maxpool_pregathered_and_gathered(dev, F, k):
    """GNN_SAGE_MAXPOOL (the north star's value max-pool): torch.max(dim=1).values, a NaN in
    the slice propagating -- vs the oracle and torch, pre-gathered and fused-gather forms."""
    from graphneuralnetwork_amd.ops import sage_aggregate, sage_gather_aggregate
    rng = np.random.default_rng(F * 31 + k)
    n, M = 4000, 257
    table = rng.standard_normal((n, F)).astype(np.float32)
    table[5, 0] = np.nan
    table[9, :] = -np.inf
    idx = rng.integers(0, n, (M, k))
    idx[0, 0] = 5
    idx[1, :] = 9
    pre = table[idx]
    ref = O.aggregator(pre, "MAXPOOL")
    tref = torch.from_numpy(pre).max(dim=1).values.numpy()
    got_p = sage_aggregate(torch.from_numpy(pre).to(dev), "MAXPOOL").cpu().numpy()
    got_g = sage_gather_aggregate(torch.from_numpy(table).to(dev), torch.from_numpy(idx).to(dev),
                                  "MAXPOOL").cpu().numpy()
    for got in (got_p, got_g):
        np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
        np.testing.assert_array_equal(got, tref)        # a max selects a value: bit-exact
    with pytest.raises(IndexError):
        sage_aggregate(torch.zeros(3, 0, F, device=dev), "MAXPOOL")


def test_maxpool_backward(dev):
    """d neigh / d table of the value max-pool vs torch autograd of .max(dim=1).values."""
    from graphneuralnetwork_amd.graphsage import Aggregator, Gathered
    gen = torch.Generator().manual_seed(4)
    n, M, k, F = 300, 200, 7, 24
    table = torch.randn(n, F, generator=gen)
    idx = torch.randint(0, n, (M, k), generator=gen)
    gy = torch.randn(M, F, generator=gen)
    t = table.to(dev).requires_grad_(True)
    (Aggregator(Gathered(t, idx.to(dev)), "MAXPOOL") * gy.to(dev)).sum().backward()
    t64 = table.double().requires_grad_(True)
    (t64[idx].max(1).values * gy.double()).sum().backward()
    np.testing.assert_allclose(t.grad.cpu().numpy(), t64.grad.numpy(), rtol=1e-5, atol=1e-6)
    x = table[idx].to(dev).requires_grad_(True)
    (Aggregator(x, "MAXPOOL") * gy.to(dev)).sum().backward()
    x64 = table[idx].double().requires_grad_(True)
    (x64.max(1).values * gy.double()).sum().backward()
    np.testing.assert_allclose(x.grad.cpu().numpy(), x64.grad.numpy(), rtol=1e-5, atol=1e-6)


def _sage_net_oracle(net, table, batch, agg):
    """oracle.graphsage_forward (GraphSAGE/GraphSAGE.py:42-53) on the batch's device maps."""
    tn = table.cpu().numpy()
    ws = [blk.weight.weight.detach().cpu().numpy() for blk in net.sage_blocks]
    dense = (net.dense.weight.detach().cpu().numpy(), net.dense.bias.detach().cpu().numpy())
    return O.graphsage_forward(tn[batch.frontier.cpu().numpy()],
                               [m.cpu().numpy() for m in batch.center_maps],
                               tn[batch.frontier_nbrs.cpu().numpy()],
                               [m.cpu().numpy() for m in batch.neigh_maps], ws, agg, False, dense)


@pytest.mark.parametrize("agg", ["MEAN", "MAXPOOL"])
def test_graphsage_sampled_forward_vs_oracle(dev, agg):
    """The [25, 10] forward on device-sampled maps (fused gather-mean, hipBLASLt / MFMA
    SageLayer GEMMs) against the numpy oracle on the same maps -- the oracle check of the
    cfg4 path at a small size (GraphSAGE/GraphSAGE.py:38-53, graph_utils.py:6)."""
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import sample_batch, symmetric_adjacency
    n, F, H = 20000, 128, 128
    s, d = rmat_edges(n, 200000, 9)
    adj = symmetric_adjacency(s, d, n, device=dev)
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu().numpy()
    seeds = torch.from_numpy(np.flatnonzero(deg > 0)[:1024]).to(dev)
    batch = sample_batch(adj, seeds, (25, 10), seed=2)
    table = torch.randn(n, F, device=dev, generator=torch.Generator(dev).manual_seed(3))
    torch.manual_seed(0)
    net = GraphSAGE(2, F, H, False, agg_func=agg, Unsupervised=False, class_size=3).to(dev).eval()
    with torch.no_grad():
        emb, logits = net(*batch.forward_args(table), None, None, None, None, None)
    ref_emb, ref_logits = _sage_net_oracle(net, table, batch, agg)
    close(emb.cpu().numpy(), ref_emb)
    close(logits.cpu().numpy(), ref_logits)


@pytest.mark.parametrize("F", [7, 64, 128, 600])
@pytest.mark.parametrize("agg", ["MEAN", "SUM", "MAXPOOL"])
def test_gather_concat_matches_separate_launches(dev, F, agg):
    """gnn_sage_gather_concat_f32: cat[table[self_idx], reduce table[idx]] in one launch equals
    the row gather + fused gather-aggregate it replaces, bit for bit, and the oracle."""
    from graphneuralnetwork_amd.ops import gather_rows, sage_gather_aggregate, sage_gather_concat
    rng = np.random.default_rng(F)
    n, M, k = 4000, 1500, 10
    table = rng.standard_normal((n, F)).astype(np.float32)
    idx = rng.integers(0, n, (M, k))
    sid = rng.integers(0, n, M)
    T, I, S = (torch.from_numpy(a).to(dev) for a in (table, idx, sid))
    got = sage_gather_concat(T, S, I, agg)
    assert torch.equal(got[:, :F], gather_rows(T, S))
    assert torch.equal(got[:, F:], sage_gather_aggregate(T, I, agg))
    np.testing.assert_array_equal(got[:, :F].cpu().numpy(), table[sid])
    ref = c_oracle.sage_gather(table, idx, agg)
    close(got[:, F:].cpu().numpy(), ref)
    bad = S.clone()
    bad[17] = n
    with pytest.raises(IndexError):
        sage_gather_concat(T, bad, I, agg)


@pytest.mark.parametrize("F", [64, 128, 600])
def test_gather_concat_argmax_as_float(dev, F):
    """GNN_SAGE_ARGMAX_F32: the concat launch's second half is torch.argmax's int64 index
    (graph_utils.py:8) as fp32 -- what torch.cat([self_feats, argmax]) promotes it to
    (GraphSAGE.py:17) -- bit for bit, incl. NaN-first and first-of-equal ties."""
    from graphneuralnetwork_amd.ops import gather_rows, sage_gather_aggregate, sage_gather_concat
    rng = np.random.default_rng(F + 1)
    n, M, k = 3000, 1200, 10
    table = rng.standard_normal((n, F)).astype(np.float32)
    table[5, :] = np.nan
    table[6, :] = table[7, :]
    idx = rng.integers(0, n, (M, k))
    idx[0, 3] = 5
    idx[1, 2], idx[1, 6] = 6, 7
    sid = rng.integers(0, n, M)
    T, I, S = (torch.from_numpy(a).to(dev) for a in (table, idx, sid))
    got = sage_gather_concat(T, S, I, "MAX")
    same = dict(rtol=0, atol=0, equal_nan=True)  # bit for bit; the NaN row may be a centre
    torch.testing.assert_close(got[:, :F], gather_rows(T, S), **same)
    arg = sage_gather_aggregate(T, I, "MAX")
    assert arg.dtype == torch.int64
    assert torch.equal(got[:, F:], arg.to(torch.float32))
    assert torch.equal(arg[0], torch.full_like(arg[0], 3))  # NaN first
    ref = torch.cat([T[S], torch.argmax(T[I], dim=1)], dim=1)  # the reference's promotion
    torch.testing.assert_close(got, ref, **same)


@pytest.mark.parametrize("agg", ["MAX", "MAXPOOL"])
def test_fused_max_layers_vs_oracle(dev, agg):
    """MAX / MAXPOOL inference on Gathered maps runs the one-launch concat + MFMA GEMM (with
    the classifier epilogue); one layer on a sampled batch against the numpy oracle
    (GraphSAGE/GraphSAGE.py:38-53, graph_utils.py:7-8; one layer: the argmax decisions are
    over the table's own values, so the oracle's float64 and the device's fp32 agree)."""
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.sampler import sample_batch
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import symmetric_adjacency
    n, F, H = 20000, 128, 128
    s, d = rmat_edges(n, 200000, 4)
    adj = symmetric_adjacency(s, d, n, device=dev)
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu().numpy()
    seeds = torch.from_numpy(np.flatnonzero(deg > 0)[:2048]).to(dev)
    batch = sample_batch(adj, seeds, (10,), seed=5)
    table = torch.randn(n, F, device=dev, generator=torch.Generator(dev).manual_seed(6))
    torch.manual_seed(1)
    net = GraphSAGE(1, F, H, False, agg_func=agg, Unsupervised=False, class_size=3).to(dev).eval()
    with torch.no_grad():
        assert net._fused_ok(net.sage_blocks[0], *batch.forward_args(table)[::2])
        emb, logits = net(*batch.forward_args(table), None, None, None, None, None)
    ref_emb, ref_logits = _sage_net_oracle(net, table, batch, agg)
    close(emb.cpu().numpy(), ref_emb)
    close(logits.cpu().numpy(), ref_logits)


def test_live_entries_touch_only_live_rows(dev):
    """gnn_sage_gather_concat_live_f32 / gnn_linear_relu_live_f32: with a device row count
    below the buffers' capacity, rows [0, live) equal the exact-size call bit for bit and the
    rows past it are neither read (garbage indices there raise no error) nor written."""
    from graphneuralnetwork_amd.ops import gcn_transform, sage_gather_concat
    g = torch.Generator(device=dev).manual_seed(8)
    n, F, H, cap, live, k = 5000, 128, 128, 3000, 1234, 10
    table = torch.randn(n, F, device=dev, generator=g)
    idx = torch.randint(0, n, (cap, k), device=dev, generator=g)
    sid = torch.randint(0, n, (cap,), device=dev, generator=g)
    idx[live:] = -7   # out of range past the count: must not be read
    sid[live:] = n + 3
    cnt = torch.tensor([live], dtype=torch.int64, device=dev)
    for agg in ("MEAN", "MAX", "MAXPOOL"):
        buf = torch.full((cap, 2 * F), 5.0, device=dev)
        sage_gather_concat(table, sid, idx, agg, check=True, out=buf, live=cnt)  # no IndexError
        ref = sage_gather_concat(table, sid[:live], idx[:live], agg)
        assert torch.equal(buf[:live], ref)
        assert bool((buf[live:] == 5.0).all())
        W = torch.randn(H, 2 * F, device=dev, generator=g) * 0.05
        y = torch.full((cap, H), -1.0, device=dev)
        gcn_transform(buf, W, relu=True, out=y, live=cnt)
        assert torch.equal(y[:live], gcn_transform(ref, W, relu=True))
        assert bool((y[live:] == -1.0).all())
    zero = torch.zeros(1, dtype=torch.int64, device=dev)
    y = torch.full((cap, H), -1.0, device=dev)
    gcn_transform(torch.randn(cap, 2 * F, device=dev), W, relu=True, out=y, live=zero)
    assert bool((y == -1.0).all())
