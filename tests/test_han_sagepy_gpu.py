"""HAN (GATConv per metapath) and GraphSAGE_Pytorch (GraphSage / SageGCN /
NeighborAggregator) drop-ins on the HIP kernels vs the reference's golden outputs
and the oracle."""
import numpy as np
import pytest
import torch

from oracle import gnn_oracle as O

pytestmark = pytest.mark.gpu


def close(a, b, rtol=1e-4):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(1.0, float(np.nanmax(np.abs(b)))) if b.size else 1.0
    np.testing.assert_allclose(a, b, rtol=rtol, atol=2e-5 * scale)


def _sd(d, prefix="sd_"):
    return {k[len(prefix):]: torch.from_numpy(np.asarray(d[k])) for k in d if k.startswith(prefix)}


def _han(golden, dev):
    from graphneuralnetwork_amd.han import HANModel
    d = golden("han")
    N, M, Fin, hid, C = (int(v) for v in d["dims"])
    net = HANModel(M, Fin, hid, C, [int(h) for h in d["heads"]], dropout=0.6)
    net.load_state_dict(_sd(d), strict=True)
    gs = []
    for m in range(M):
        A = torch.zeros(N, N)
        A[torch.from_numpy(d[f"g{m}_row"]).long(), torch.from_numpy(d[f"g{m}_col"]).long()] = 1
        gs.append(A.to(dev))
    return d, net.to(dev), gs, torch.from_numpy(d["h"]).to(dev)


def test_han_matches_reference(golden, dev):
    d, net, gs, h = _han(golden, dev)
    net.eval()
    with torch.no_grad():
        close(net.layers[0](gs, h).cpu().numpy(), d["layer0"])
        close(net(gs, h).cpu().numpy(), d["logits"])


def test_han_gatconv_with_classes_vs_oracle(dev):
    from graphneuralnetwork_amd.han import GATConv
    torch.manual_seed(3)
    N, Fin, hid, heads, C = 200, 16, 8, 3, 5
    A = (torch.rand(N, N) < 0.05).float()
    A.fill_diagonal_(1)
    conv = GATConv(Fin, hid, 0.5, heads, num_class=C).eval()
    h = torch.randn(N, Fin)
    with torch.no_grad():
        y = conv.to(dev)(h.to(dev), A.to(dev)).cpu().numpy()
    hp = [(m.W.detach().cpu().numpy(), m.a.detach().cpu().numpy()) for m in conv.attentions]
    ref = O.han_gatconv(h.numpy(), A.numpy(), hp, 0.2,
                        (conv.out_att.W.detach().cpu().numpy(), conv.out_att.a.detach().cpu().numpy()))
    close(y, ref)


def test_han_trains(golden, dev):
    d, net, gs, h = _han(golden, dev)
    net.train()
    opt = torch.optim.SGD(net.parameters(), lr=0.01)
    y = torch.randint(0, int(d["dims"][4]), (h.shape[0],), device=dev)
    losses = []
    for _ in range(5):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(net(gs, h), y)
        loss.backward()
        assert all(torch.isfinite(p.grad).all() for p in net.parameters() if p.grad is not None)
        opt.step()
        losses.append(loss.item())
    assert np.isfinite(losses).all()


def _sagepy(golden, dev):
    from graphneuralnetwork_amd.graphsage_pytorch import GraphSage
    d = golden("sagepy")
    Fin, B, h0, h1, k0, k1 = (int(v) for v in d["dims"])
    net = GraphSage(Fin, [h0, h1], [k0, k1])
    net.load_state_dict(_sd(d), strict=True)
    return d, net.to(dev)


def test_graphsage_pytorch_matches_reference(golden, dev):
    from graphneuralnetwork_amd.graphsage_pytorch import NeighborAggregator, SageGCN
    d, net = _sagepy(golden, dev)
    Fin, B, h0, h1, k0, k1 = (int(v) for v in d["dims"])
    feats = [torch.from_numpy(d[f"X{i}"]).to(dev) for i in range(3)]
    with torch.no_grad():
        close(net(feats).cpu().numpy(), d["y"])
        layer = SageGCN(Fin, 12, aggr_neighbor_method="sum", aggr_hidden_method="concat")
        layer.load_state_dict(_sd(d, "sumcat_sd_"), strict=True)
        nb = feats[1].view(B, k0, Fin)
        close(layer.to(dev)(feats[0], nb).cpu().numpy(), d["sumcat_y"])
        agg = NeighborAggregator(Fin, 7, use_bias=True)
        agg.load_state_dict(_sd(d, "biasmean_sd_"), strict=True)
        close(agg.to(dev)(nb).cpu().numpy(), d["biasmean_y"])


@pytest.mark.parametrize("method", ["mean", "sum"])
def test_sage_sum_and_mean_kernels_vs_oracle(dev, method):
    from graphneuralnetwork_amd.ops import sage_aggregate, sage_gather_aggregate
    rng = np.random.default_rng(5)
    nb = rng.standard_normal((333, 7, 36)).astype(np.float32)
    kind = method.upper()
    ref = nb.astype(np.float64).mean(1) if method == "mean" else nb.astype(np.float64).sum(1)
    close(sage_aggregate(torch.from_numpy(nb).to(dev), kind).cpu().numpy(), ref)
    table = rng.standard_normal((90, 36)).astype(np.float32)
    idx = rng.integers(0, 90, (333, 7))
    t = table[idx].astype(np.float64)
    ref = t.mean(1) if method == "mean" else t.sum(1)
    out = sage_gather_aggregate(torch.from_numpy(table).to(dev), torch.from_numpy(idx).to(dev), kind)
    close(out.cpu().numpy(), ref)


def test_graphsage_pytorch_sampled_gathered_path(dev):
    """multihop_sampling on the device + Gathered hops == pre-gathered hops == oracle; and the
    table gradient of the fused path matches torch autograd of the gathered form."""
    from graphneuralnetwork_amd.graphsage_pytorch import GraphSage, multihop_sampling
    from graphneuralnetwork_amd.graphsage import Gathered
    from graphneuralnetwork_amd.sampler import symmetric_adjacency
    rng = np.random.default_rng(9)
    n, Fin, nbrs = 2000, 24, [6, 4]
    s, t = rng.integers(0, n, 20000), rng.integers(0, n, 20000)
    adj = symmetric_adjacency(s, t, n, device=dev)
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu().numpy()
    src = torch.from_numpy(np.flatnonzero(deg > 0)[:50]).to(dev)
    hops = multihop_sampling(src, nbrs, adj, seed=4)
    assert [h.numel() for h in hops] == [50, 300, 1200]
    rp, col = adj.rowptr.cpu().numpy(), adj.col.cpu().numpy()
    for a, b, k in zip(hops[:-1], hops[1:], nbrs):
        for u, vs in zip(a.cpu().numpy(), b.view(-1, k).cpu().numpy()):
            assert set(vs) <= set(col[rp[u]:rp[u + 1]])
    torch.manual_seed(0)
    net = GraphSage(Fin, [16, 3], nbrs).to(dev)
    table = torch.randn(n, Fin, device=dev, requires_grad=True)
    y_g = net([Gathered(table, h) for h in hops])
    y_d = net([table[h] for h in hops])
    close(y_g.detach().cpu().numpy(), y_d.detach().cpu().numpy())
    layers = [(g.weight.detach().cpu().numpy(), g.aggregator.weight.detach().cpu().numpy())
              for g in net.gcn]
    ref = O.graphsage_tree([table.detach().cpu().numpy()[h.cpu().numpy()] for h in hops], layers,
                           nbrs)
    close(y_g.detach().cpu().numpy(), ref)
    gy = torch.randn_like(y_g)
    (g1,) = torch.autograd.grad((y_g * gy).sum(), table)
    (g2,) = torch.autograd.grad((y_d * gy).sum(), table)
    close(g1.cpu().numpy(), g2.cpu().numpy())


def test_han_layer_batched_metapaths_match(golden, dev, monkeypatch):
    """The inference HANLayer runs all metapaths as ONE block-diagonal aggregation launch;
    it equals the per-metapath GATConv path (and so the reference), and a metapath graph
    with an edgeless row falls back to the per-metapath path."""
    from graphneuralnetwork_amd import han
    d, net, gs, h = _han(golden, dev)
    net.eval()
    with torch.no_grad():
        batched = net(gs, h)
        assert net.layers[0]._block_cache[1] is not None
        monkeypatch.setattr(han, "BATCH_METAPATHS", False)
        single = net(gs, h)
    close(batched.cpu().numpy(), single.cpu().numpy(), rtol=1e-5)
    close(batched.cpu().numpy(), d["logits"])
    monkeypatch.setattr(han, "BATCH_METAPATHS", True)
    g0 = gs[0].clone()
    g0[5, :] = 0                                  # an edgeless row in metapath 0
    with torch.no_grad():
        y = net.layers[0]([g0] + gs[1:], h)
        assert net.layers[0]._block_cache[1] is None
        monkeypatch.setattr(han, "BATCH_METAPATHS", False)
        y0 = net.layers[0]([g0] + gs[1:], h)
    close(y.cpu().numpy(), y0.cpu().numpy(), rtol=1e-5)
