"""Parity at BASELINE.json's full sizes (north star 10M / 100M at F=128 and F=256; GAT cfg3).

The oracle cannot run the whole graph in seconds, so each case checks
  * an exact float64 restatement (oracle/spmm_oracle.c, oracle.gnn_oracle.gat_csr) on a row
    sample that always contains the highest-degree rows (the long-row / fix-up path, the
    187,554-edge hub at 10M) plus random rows of every class, and
  * a size-independent property over ALL rows: the checksum of checksums
    1^T (A X) v = (1^T A) (X v)  (linearity; column sums of A computed in float64).
Tolerance (north_star): fp32 within 1e-4 relative.
"""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from oracle import gnn_oracle as O

pytestmark = pytest.mark.gpu


def close(a, b, rtol=1e-4):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(1.0, float(np.abs(b).max()))
    np.testing.assert_allclose(a, b, rtol=rtol, atol=1e-5 * scale)


@pytest.fixture(scope="module")
def ns_graph():
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n = 10_000_000
    s, d = rmat_edges(n, 100_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    host = {k: getattr(g, k).cpu().numpy() for k in ("rowptr", "col", "val")}
    yield g, host
    del g
    torch.cuda.empty_cache()


def _sample_rows(rowptr, n, k, seed):
    deg = np.diff(rowptr)
    rng = np.random.default_rng(seed)
    return np.unique(np.concatenate([rng.choice(n, k, replace=False), np.argsort(-deg)[:32],
                                     np.flatnonzero(deg == 1)[:64]]))


@pytest.mark.parametrize("F", [128, 256])
def test_north_star_spmm_full_size(ns_graph, F):
    from graphneuralnetwork_amd.ops import spmm_forward
    g, h = ns_graph
    assert g.nnz == 206_948_698 and g.n_rows == 10_000_000
    dev = g.rowptr.device
    X = torch.randn(g.n_rows, F, device=dev, generator=torch.Generator(dev).manual_seed(F))
    b = torch.randn(F, device=dev, generator=torch.Generator(dev).manual_seed(1))
    Y = spmm_forward(g, X, b)
    rows = _sample_rows(h["rowptr"], g.n_rows, 2000, F)
    Xn = X.cpu().numpy()
    bn = b.cpu().numpy()
    ref = np.concatenate([c_oracle.spmm_csr(h["rowptr"], h["col"], h["val"], Xn, bn, r, r + 1)
                          for r in rows])
    close(Y[torch.from_numpy(rows).to(dev)].cpu().numpy(), ref)
    # checksum of checksums over all 10M rows: 1^T (A X + 1 b^T) v == (1^T A)(X v) + n (b . v)
    v = np.random.default_rng(2).standard_normal(F)
    lhs = float((Y.double() @ torch.from_numpy(v).to(dev)).sum())
    colsum_a = np.bincount(h["col"], weights=h["val"].astype(np.float64), minlength=g.n_cols)
    rhs = float(colsum_a @ (Xn.astype(np.float64) @ v)) + g.n_rows * float(bn.astype(np.float64) @ v)
    scale = float(np.abs(colsum_a) @ np.abs(Xn.astype(np.float64) @ v))
    assert abs(lhs - rhs) <= 1e-4 * scale, (lhs, rhs, scale)


def test_gat_cfg3_full_size():
    """BASELINE configs[2]: 8-head GAT (dense and sparse semantics) over the 1M / 10M graph."""
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.ops import GAT_DENSE, GAT_SPARSE, gat_aggregate, gat_project
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, H, fh, Fin = 1_000_000, 8, 8, 64
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    gen = torch.Generator(dev).manual_seed(0)
    X = torch.randn(n, Fin, device=dev, generator=gen)
    W = torch.randn(Fin, H * fh, device=dev, generator=gen) * 0.2
    a_s = torch.randn(H * fh, device=dev, generator=gen) * 0.3
    a_d = torch.randn(H * fh, device=dev, generator=gen) * 0.3
    wh, el, er = gat_project(X, W, H, fh, a_s, a_d)
    whn = X.cpu().double().numpy() @ W.cpu().double().numpy()
    close(wh.cpu().numpy(), whn)
    el_o, er_o = O.gat_logits(whn, H, fh, a_s.cpu().numpy(), a_d.cpu().numpy())
    close(el.cpu().numpy(), el_o)
    close(er.cpu().numpy(), er_o)
    rowptr, col = g.rowptr.cpu().numpy(), g.col.cpu().numpy()
    rows = _sample_rows(rowptr, n, 3000, 7)
    sub_ptr = np.concatenate([[0], np.cumsum(np.diff(rowptr)[rows])])
    sub_col = np.concatenate([col[rowptr[r]:rowptr[r + 1]] for r in rows])
    gg = CsrGraph(g.rowptr, g.col, torch.ones_like(g.val), n, n)
    for mode, sparse in ((GAT_DENSE, False), (GAT_SPARSE, True)):
        out = gat_aggregate(gg, wh, el, er, H, fh, 0.2, mode)
        ref = O.gat_csr(sub_ptr, sub_col, whn, el_o[rows], er_o, H, fh, 0.2, sparse)
        close(out[torch.from_numpy(rows).to(dev)].cpu().numpy(), ref)
        # every row's attention weights sum to one: aggregating Wh = 1 gives exactly 1
        ones = torch.ones_like(wh)
        o1 = gat_aggregate(gg, ones, el, er, H, fh, 0.2, mode)
        assert float((o1 - 1).abs().max()) < 1e-5


@pytest.mark.parametrize("agg", ["MEAN"])
def test_graphsage_cfg4_full_size(agg):
    """BASELINE configs[3]: the device-sampled [25, 10] batch of 8192 seeds (degree >= 1) on
    the 10M / 100M R-MAT adjacency, the drop-in GraphSAGE(2, 128, 128, MEAN) forward on a
    10M x 128 table (5.1 GB: row offsets pass 2^32 bytes), against the numpy oracle
    (GraphSAGE/GraphSAGE.py:38-53, graph_utils.py:6) on the SAME maps: every seed's embedding
    and logits within 1e-4, plus a layer-0 gather-mean sample over the table's last rows."""
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.ops import sage_gather_aggregate
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
    assert batch.neigh_map.shape == (8192, 25) and batch.frontier_nbrs.shape[1] == 10
    torch.manual_seed(0)
    net = GraphSAGE(2, F, F, False, agg_func=agg, Unsupervised=False, class_size=3).to(dev).eval()
    with torch.no_grad():
        emb, logits = net(*batch.forward_args(table), None, None, None, None, None)
    tn = table.cpu().numpy()
    ws = [blk.weight.weight.detach().cpu().numpy() for blk in net.sage_blocks]
    dense = (net.dense.weight.detach().cpu().numpy(), net.dense.bias.detach().cpu().numpy())
    ref_emb, ref_logits = O.graphsage_forward(
        tn[batch.frontier.cpu().numpy()], [m.cpu().numpy() for m in batch.center_maps],
        tn[batch.frontier_nbrs.cpu().numpy()], [m.cpu().numpy() for m in batch.neigh_maps],
        ws, agg, False, dense)
    close(emb.cpu().numpy(), ref_emb)
    close(logits.cpu().numpy(), ref_logits)
    # layer-0 gather-mean over index rows that include the table's last rows (byte offsets
    # above 2^32: row 8,388,608 onward at F = 128)
    rng = np.random.default_rng(5)
    idx = rng.integers(0, n, (4096, 10))
    idx[:64] = n - 1 - np.arange(640).reshape(64, 10)
    idx[64:96] = (1 << 32) // (4 * F) + np.arange(320).reshape(32, 10)
    got = sage_gather_aggregate(table, torch.from_numpy(idx).to(dev), agg).cpu().numpy()
    close(got, c_oracle.sage_gather(tn, idx, agg))
    assert int(batch.frontier.max()) >= (1 << 32) // (4 * F)  # sampled rows past 2^32 bytes too


# ---------------------------------------------------------------------------------------------
# The variants bench.py times, pinned at full size: the
# column-degree-ordered Graph_conv_layer (A P^T, support rows scattered by the MFMA transform,
# hub rows read in place by the XCD-sliced SpMM) at cfg2 and at the north star; the GAT heads
# layer through _ordered (gnn_gat_project_rows_f32 + order.graph) at cfg3; the GraphSAGE forward
# over sampler.degree_ordered at cfg4. Each against the oracle on a row sample holding the 32
# hottest rows, plus an all-row checksum; each asserts the ordered plan was the one taken.
# ---------------------------------------------------------------------------------------------
def _sub_csr(rowptr, col, val, rows):
    """The CSR of the sampled rows with their columns renumbered into `need` (the distinct
    columns they gather): (sub_rowptr, sub_col, sub_val, need)."""
    deg = np.diff(rowptr)[rows]
    sub_ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    sub_col = np.concatenate([col[rowptr[r]:rowptr[r + 1]] for r in rows]).astype(np.int64)
    sub_val = np.concatenate([val[rowptr[r]:rowptr[r + 1]] for r in rows])
    need, inv = np.unique(sub_col, return_inverse=True)
    return sub_ptr, inv.astype(np.int32), sub_val, need


def _assert_colorder_taken(g):
    """The layer ran over the cached column-degree order with the XCD-sliced plan reading the
    hub rows in place (XcdHubPlan.prefix), as bench.py's headline does."""
    from graphneuralnetwork_amd import ops
    assert ("_colorder",) in g._plans
    og = g._plans[("_colorder",)].graph
    xps = [p for k, p in og._plans.items() if isinstance(k, tuple) and k[0] == "_xcd"]
    assert xps and all(p is not None and p.prefix for p in xps)
    assert ops.XCD_DIRECT and ops.DEGREE_ORDER and ops.SPMM_TASKS


def _gcn_layer_full_size(g, h, F, seed):
    from graphneuralnetwork_amd.gcn import Graph_conv_layer
    dev = g.rowptr.device
    gen = torch.Generator(dev).manual_seed(seed)
    layer = Graph_conv_layer(F, F).to(dev).eval()
    with torch.no_grad():
        layer.bias.copy_(torch.randn(F, device=dev, generator=gen))
    X = torch.randn(g.n_rows, F, device=dev, generator=gen)
    with torch.no_grad():
        Y = layer(X, g)
    _assert_colorder_taken(g)
    W = layer.dense.weight.detach().double().cpu().numpy()
    bn = layer.bias.detach().cpu().numpy()
    rows = _sample_rows(h["rowptr"], g.n_rows, 2000, seed)
    sp, sc, sv, need = _sub_csr(h["rowptr"], h["col"], h["val"], rows)
    support = (X[torch.from_numpy(need).to(dev)].double().cpu().numpy() @ W.T).astype(np.float32)
    ref = c_oracle.spmm_csr(sp, sc, sv, support, bn)
    close(Y[torch.from_numpy(rows).to(dev)].cpu().numpy(), ref)
    # checksum of checksums over every row: 1^T (A X W^T + 1 b^T) v = (1^T A)(X (W^T v)) + n b.v
    v = np.random.default_rng(seed + 1).standard_normal(F)
    lhs = float((Y.double() @ torch.from_numpy(v).to(dev)).sum())
    xu = (X.double() @ torch.from_numpy(W.T @ v).to(dev)).cpu().numpy()
    colsum_a = np.bincount(h["col"], weights=h["val"].astype(np.float64), minlength=g.n_cols)
    rhs = float(colsum_a @ xu) + g.n_rows * float(bn.astype(np.float64) @ v)
    scale = float(np.abs(colsum_a) @ np.abs(xu))
    assert abs(lhs - rhs) <= 1e-4 * scale, (lhs, rhs, scale)


@pytest.mark.parametrize("F", [128, 256])
def test_bench_variant_gcn_layer_north_star(ns_graph, F):
    """bench.py's north-star line (F=128) and the cfg5 layer at one GPU (F=256):
    Graph_conv_layer(F, F).eval() over the 10M / 207M graph (GCN/GCN.py:41-47), through the
    column-degree order with default knobs (F=256: the one-launch 256-column transform)."""
    g, h = ns_graph
    _gcn_layer_full_size(g, h, F, 11 + F)


@pytest.fixture(scope="module")
def cfg2_graph():
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n = 1_000_000
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    host = {k: getattr(g, k).cpu().numpy() for k in ("rowptr", "col", "val")}
    yield g, host
    del g
    torch.cuda.empty_cache()


def test_bench_variant_gcn_layer_cfg2(cfg2_graph):
    """bench.py's headline graph (BASELINE configs[1], nnz 20,073,500): the same layer."""
    g, h = cfg2_graph
    assert g.nnz == 20_073_500
    _gcn_layer_full_size(g, h, 128, 12)


def test_bench_variant_gcn_spmm_cfg2_all_rows(cfg2_graph):
    """The headline step itself (bench.py run_gcn: spmm_forward over column_order(g).graph with
    X = the support in that row order) against the C oracle on EVERY row of cfg2."""
    from graphneuralnetwork_amd.ops import column_order, spmm_forward
    g, h = cfg2_graph
    dev = g.rowptr.device
    F = 128
    gen = torch.Generator(dev).manual_seed(3)
    bias = torch.randn(F, device=dev, generator=gen)
    X = torch.randn(g.n_cols, F, device=dev, generator=gen)
    order = column_order(g, F)
    assert order is not None
    Y = spmm_forward(order.graph, X, bias)
    _assert_colorder_taken(g)
    # X holds the support in the new order: row j of X is old column perm[j]
    Xold = X[order.inv].cpu().numpy()
    ref = c_oracle.spmm_csr(h["rowptr"], h["col"], h["val"], Xold, bias.cpu().numpy())
    close(Y.cpu().numpy(), ref)


@pytest.mark.parametrize("model", ["GAT", "SpGAT"])
def test_bench_variant_gat_heads_cfg3(model):
    """bench.py's cfg3 line: the 8-head layer of GAT(64, 8, ., 8) at inference (GATBase._heads ->
    _ordered: gnn_gat_project_rows_f32 writing Wh / er in the column-degree order, the
    aggregation over order.graph reading the hub rows in place; GAT/models/layers.py:22-37,
    GAT.py:16) on the 1M / 10M graph, against the oracle on a row sample with the 32 hottest
    rows, plus every row's attention mass (Wh = 1 aggregates to ELU(1))."""
    from graphneuralnetwork_amd import gat as gat_mod
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, H, fh, Fin = 1_000_000, 8, 8, 64
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    torch.manual_seed(0)
    net = getattr(gat_mod, model)(Fin, fh, 7, 0.6, 0.2, H).to(dev).eval()
    X = torch.randn(n, Fin, device=dev, generator=torch.Generator(dev).manual_seed(4))
    with torch.no_grad():
        out = net._heads(X, g)
    assert ("_colorder",) in g._plans
    og = g._plans[("_colorder",)].graph
    hubs = [p for k, p in og._plans.items() if isinstance(k, tuple) and k[0] == "_hub"]
    assert hubs and all(p.prefix for p in hubs)  # Wh / er hub rows read in place
    W = torch.cat([m.W for m in net.attentions], 1).detach().double().cpu().numpy()
    a = [m.a.detach().reshape(-1).cpu().numpy() for m in net.attentions]
    a_s = np.concatenate([x[:fh] for x in a])
    a_d = np.concatenate([x[fh:] for x in a])
    rowptr, col = g.rowptr.cpu().numpy(), g.col.cpu().numpy()
    rows = _sample_rows(rowptr, n, 3000, 9)
    sp, sc, _, need = _sub_csr(rowptr, col, np.ones(col.size, np.float32), rows)
    Xn_need = X[torch.from_numpy(need).to(dev)].double().cpu().numpy()
    Xn_rows = X[torch.from_numpy(rows).to(dev)].double().cpu().numpy()
    wh_need = Xn_need @ W
    el_rows, _ = O.gat_logits(Xn_rows @ W, H, fh, a_s, a_d)
    _, er_need = O.gat_logits(wh_need, H, fh, a_s, a_d)
    ref = O.gat_csr(sp, sc, wh_need, el_rows, er_need, H, fh, 0.2, model == "SpGAT")
    ref = np.where(ref > 0, ref, np.expm1(np.minimum(ref, 0)))  # concat heads: ELU
    close(out[torch.from_numpy(rows).to(dev)].cpu().numpy(), ref)
    assert bool(torch.isfinite(out).all())


def test_bench_variant_graphsage_cfg4_degree_ordered():
    """bench.py's cfg4 line: the dataset relabelled by sampler.degree_ordered, the device-sampled
    [25, 10] batch of 8192 seeds, GraphSAGE(2, 128, 128, MEAN).eval() (GraphSAGE.py:38-53):
    the relabelled adjacency is P A P^T exactly (neighbour sets of sampled rows, bit-exact), and
    the forward matches the oracle on the same maps within 1e-4."""
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import degree_ordered, sample_batch, symmetric_adjacency
    dev = torch.device("cuda:0")
    n, F = 10_000_000, 128
    s, d = rmat_edges(n, 100_000_000, 0)
    adj0 = symmetric_adjacency(s, d, n, device=dev)
    del s, d
    adj, _, order = degree_ordered(adj0)
    # structure: new row i lists inv[old neighbours of perm[i]], ascending
    rp0, c0 = adj0.rowptr.cpu().numpy(), adj0.col.cpu().numpy()
    rp1, c1 = adj.rowptr.cpu().numpy(), adj.col.cpu().numpy()
    perm, inv = order.perm.cpu().numpy(), order.inv.cpu().numpy()
    deg1 = np.diff(rp1)
    assert np.all(deg1[:-1] >= deg1[1:])  # degree order, hottest first
    chk = np.unique(np.concatenate([np.arange(32), np.random.default_rng(3).choice(n, 2000)]))
    for i in chk:
        o = perm[i]
        want = np.sort(inv[c0[rp0[o]:rp0[o + 1]]])
        np.testing.assert_array_equal(c1[rp1[i]:rp1[i + 1]], want)
    del adj0, rp0, c0
    gen = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(n, F, device=dev, generator=gen)
    deg = adj.rowptr[1:] - adj.rowptr[:-1]
    cand = torch.nonzero(deg > 0).view(-1)
    seeds = cand[torch.randperm(cand.numel(), device=dev, generator=gen)[:8192]]
    batch = sample_batch(adj, seeds, (25, 10), seed=0)
    torch.manual_seed(0)
    net = GraphSAGE(2, F, F, False, agg_func="MEAN", Unsupervised=False, class_size=3).to(dev).eval()
    with torch.no_grad():
        emb, logits = net(*batch.forward_args(table), None, None, None, None, None)
    tn = table.cpu().numpy()
    ws = [blk.weight.weight.detach().cpu().numpy() for blk in net.sage_blocks]
    dense = (net.dense.weight.detach().cpu().numpy(), net.dense.bias.detach().cpu().numpy())
    ref_emb, ref_logits = O.graphsage_forward(
        tn[batch.frontier.cpu().numpy()], [m.cpu().numpy() for m in batch.center_maps],
        tn[batch.frontier_nbrs.cpu().numpy()], [m.cpu().numpy() for m in batch.neigh_maps],
        ws, "MEAN", False, dense)
    close(emb.cpu().numpy(), ref_emb)
    close(logits.cpu().numpy(), ref_logits)
    # every sampled neighbour is a true neighbour in the relabelled graph
    fr = batch.frontier.cpu().numpy()
    nb = batch.frontier_nbrs.cpu().numpy()
    for r in range(0, fr.size, max(1, fr.size // 500)):
        assert np.isin(nb[r], c1[rp1[fr[r]]:rp1[fr[r] + 1]]).all()


@pytest.mark.parametrize("order", ["degree", "natural"])
@pytest.mark.parametrize("model,drop", [("GAT", 0.0), ("GAT", 0.3), ("SpGAT", 0.0),
                                        ("SpGAT", 0.3)])
def test_gat_training_block_cfg3_vs_oracle(model, drop, order, monkeypatch):
    """bench.py's cfg3 training step at full size: the 8-head attention
    block of GAT / SpGAT(64, 8, ., 8) in train mode (GATBase._heads: _ProjectFn on the MFMA
    transform, _GatLayerFn's fused forward with per-row LSE stats, the two-pass HIP backward:
    prep + row pass, recomputing node pass over A itself) on the 1M / 10M graph, forward +
    loss.backward() for loss = sum(out * gy), against the float64 C restatement of the block
    and its gradients over all 20M edges (oracle_gat_block_grad, pinned by the reference's own
    autograd in tests/test_oracle_golden.py): the block output, every head's dW and da, and dX
    on every row (the 32 hottest rows included), with and without dropout (the oracle re-derives
    the kernels' (seed, edge, head) masks). Replaces the HIP-vs-HIP check
    (test_gat_gpu.py::test_gat_backward_two_pass_matches_three_pass_cfg3). order "degree": the
    block over P A P^T with X in that order, as GATBase.forward trains (ops.gat_train_order);
    "natural": over A itself.
    Reference: GAT/models/layers.py:22-37, :54-64, :94-131. Tolerance 1e-4 relative."""
    from graphneuralnetwork_amd import gat as gat_mod
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, H, fh, Fin, seed = 1_000_000, 8, 8, 64, 0x5EED_0F_CF63
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    if order == "degree":
        from graphneuralnetwork_amd.ops import gat_train_order
        o = gat_train_order(g, H, fh)
        assert o is not None and o.graph.symmetric
        g = o.graph
    torch.manual_seed(1)
    net = getattr(gat_mod, model)(Fin, fh, 7, drop, 0.2, H).to(dev).train()
    monkeypatch.setattr(gat_mod, "_dropout_seed", lambda: seed)
    gen = torch.Generator(dev).manual_seed(5)
    X = torch.randn(n, Fin, device=dev, generator=gen).requires_grad_(True)
    gy = torch.randn(n, H * fh, device=dev, generator=gen)
    out = net._heads(X, g)
    out.backward(gy)
    W = torch.cat([m.W for m in net.attentions], 1).detach().cpu().numpy()
    a = [m.a.detach().reshape(-1).cpu().numpy() for m in net.attentions]
    a_s = np.concatenate([x[:fh] for x in a])
    a_d = np.concatenate([x[fh:] for x in a])
    rowptr, col = g.rowptr.cpu().numpy(), g.col.cpu().numpy()
    r = c_oracle.gat_block_grad(rowptr, col, X.detach().cpu().numpy(), W, a_s, a_d,
                                gy.cpu().numpy(), H, fh, 0.2, model == "SpGAT", drop_p=drop,
                                drop_seed=seed)
    dW = torch.cat([m.W.grad for m in net.attentions], 1).cpu().numpy()
    da = np.stack([m.a.grad.reshape(-1).cpu().numpy() for m in net.attentions])
    dx = X.grad.cpu().numpy()
    hot = np.argsort(-np.diff(rowptr))[:32]
    da_ref = np.concatenate([r["da_src"].reshape(H, fh), r["da_dst"].reshape(H, fh)], axis=1)
    da_slack = np.concatenate([r["slack_da_src"].reshape(H, fh),
                               r["slack_da_dst"].reshape(H, fh)], axis=1)
    # tolerance: fp32 within 1e-4 relative -- element-wise for the block output and dX (plus
    # an absolute 1e-5 of the tensor's largest entry); dW and da are sums over all 1M rows of
    # terms that largely cancel (a softmax gradient sums to zero over a row), held to 1e-4 of
    # the tensor's largest entry. On top, each element may move by the oracle's kink slack:
    # LeakyReLU' jumps from 1 to 0.2 at t = 0, and an edge whose t_ij = el_i + er_j is within
    # fp32 rounding of 0 may take either branch (a handful of the 160M (edge, head) pairs)
    cases = {"out": (out.detach().cpu().numpy(), r["out"], 0.0, False),
             "dx": (dx, r["dx"], r["slack_dx"], False),
             "dx_hot": (dx[hot], r["dx"][hot], r["slack_dx"][hot], False),
             "dW": (dW, r["dW"], r["slack_dW"], True), "da": (da, da_ref, da_slack, True)}
    kinks = int((r["kink_del"] > 0).sum())
    report, bad = [], []
    for k, (hip, ref, slack, normwise) in cases.items():
        scale = float(np.abs(ref).max())
        tol = (1e-4 * scale if normwise else 1e-4 * np.abs(ref) + 1e-5 * max(1.0, scale)) + slack
        excess = np.abs(hip - ref) - tol
        report.append(f"{k} {float(np.abs(hip - ref).max()) / scale:.2e}")
        if not normwise and np.ndim(slack) == 2:  # rows no kink edge reaches
            clean = np.abs(slack).max(1) == 0
            if clean.any():
                report.append(f"{k}[no kink] "
                              f"{float(np.abs(hip - ref)[clean].max()) / scale:.2e}")
        if excess.max() > 0:
            bad.append((k, float(excess.max()), np.unravel_index(excess.argmax(), excess.shape)))
    print(f"{model} {order} order, dropout {drop}: kink (row, head) pairs {kinks}; max |hip - oracle| / "
          "max |oracle|: " + ", ".join(report))
    assert not bad, bad


def _check_layer(name, hip):
    """hip: {name: (fp32 result, float64 oracle, kink slack, normwise)}: elementwise 1e-4 relative
    (+1e-5 of the max) or normwise 1e-4 of the max, plus the oracle's LeakyReLU-kink slack."""
    report, bad = [], []
    for k, (h, ref, slack, normwise) in hip.items():
        scale = float(np.abs(ref).max())
        tol = (1e-4 * scale if normwise else 1e-4 * np.abs(ref) + 1e-5 * max(1.0, scale)) + slack
        excess = np.abs(h - ref) - tol
        report.append(f"{k} {float(np.abs(h - ref).max()) / scale:.2e}")
        if excess.max() > 0:
            bad.append((k, float(excess.max())))
    print(f"{name}: " + ", ".join(report))
    assert not bad, (name, bad)


@pytest.mark.parametrize("model", ["GAT", "SpGAT"])
def test_gat_model_training_cfg3_vs_oracle(model):
    """The whole GAT model's training step at cfg3 size (GAT/SpGAT(64, 8, 7, ., 8); GAT.py:14-18,
    train_eval.py:72-76), as GATBase.forward runs it: over P A P^T, the 8-head block, then the
    7-class out_att (zero-padded to 8 features for the two-pass backward, its dW / da on the
    narrow / tiny gemm_tn kernels), ELU. Each layer against the float64 oracle given the same
    inputs: out_att with the block's fp32 output as its input and the loss gradient, the block
    with the gradient out_att handed back. Dropout 0 (F.dropout's torch RNG is not restated;
    the block's dropout is pinned by test_gat_training_block_cfg3_vs_oracle)."""
    from graphneuralnetwork_amd import gat as gat_mod
    from graphneuralnetwork_amd.ops import gat_train_order
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    dev = torch.device("cuda:0")
    n, H, fh, Fin, C = 1_000_000, 8, 8, 64, 7
    s, d = rmat_edges(n, 10_000_000, 0)
    g = gcn_adjacency(torch.from_numpy(s).to(dev), torch.from_numpy(d).to(dev), n)
    del s, d
    g = gat_train_order(g, H, fh).graph
    torch.manual_seed(2)
    net = getattr(gat_mod, model)(Fin, fh, C, 0.0, 0.2, H).to(dev).train()
    gen = torch.Generator(dev).manual_seed(6)
    X = torch.randn(n, Fin, device=dev, generator=gen).requires_grad_(True)
    gy = torch.randn(n, C, device=dev, generator=gen)
    x1 = net._heads(X, g)
    x1.retain_grad()
    out = net.out_att(x1, g, activation="elu")
    out.backward(gy)
    rowptr, col = g.rowptr.cpu().numpy(), g.col.cpu().numpy()
    sparse = model == "SpGAT"
    # out_att: 1 head x 7, input the block's fp32 output
    W2 = net.out_att.W.detach().cpu().numpy()
    a2 = net.out_att.a.detach().reshape(-1).cpu().numpy()
    r2 = c_oracle.gat_block_grad(rowptr, col, x1.detach().cpu().numpy(), W2, a2[:C], a2[C:],
                                 gy.cpu().numpy(), 1, C, 0.2, sparse)
    da2 = net.out_att.a.grad.reshape(-1).cpu().numpy()
    _check_layer(f"{model} out_att", {
        "out": (out.detach().cpu().numpy(), r2["out"], 0.0, False),
        "dx": (x1.grad.cpu().numpy(), r2["dx"], r2["slack_dx"], False),
        "dW": (net.out_att.W.grad.cpu().numpy(), r2["dW"], r2["slack_dW"], True),
        "da": (da2, np.concatenate([r2["da_src"], r2["da_dst"]]),
               np.concatenate([r2["slack_da_src"], r2["slack_da_dst"]]), True)})
    # the 8-head block with the gradient out_att handed back
    W1 = torch.cat([m.W for m in net.attentions], 1).detach().cpu().numpy()
    a1 = [m.a.detach().reshape(-1).cpu().numpy() for m in net.attentions]
    r1 = c_oracle.gat_block_grad(rowptr, col, X.detach().cpu().numpy(), W1,
                                 np.concatenate([x[:fh] for x in a1]),
                                 np.concatenate([x[fh:] for x in a1]), x1.grad.cpu().numpy(), H,
                                 fh, 0.2, sparse)
    da1 = np.stack([m.a.grad.reshape(-1).cpu().numpy() for m in net.attentions])
    _check_layer(f"{model} heads", {
        "out": (x1.detach().cpu().numpy(), r1["out"], 0.0, False),
        "dx": (X.grad.cpu().numpy(), r1["dx"], r1["slack_dx"], False),
        "dW": (torch.cat([m.W.grad for m in net.attentions], 1).cpu().numpy(), r1["dW"],
               r1["slack_dW"], True),
        "da": (da1, np.concatenate([r1["da_src"].reshape(H, fh), r1["da_dst"].reshape(H, fh)], 1),
               np.concatenate([r1["slack_da_src"].reshape(H, fh),
                               r1["slack_da_dst"].reshape(H, fh)], 1), True)})
