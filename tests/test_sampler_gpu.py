"""Device neighbour sampler (GraphSAGE/data_utils.py:82-117 semantics) and the
fused Gathered forward path."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _adj(dev, n=3000, e=20000, seed=0):
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import symmetric_adjacency
    s, d = rmat_edges(n, e, seed)
    return symmetric_adjacency(s, d, n, device=dev)


@pytest.mark.parametrize("k", [1, 10, 16, 25, 32, 40])  # register paths (<= 16, <= 32), generic
def test_sample_rules(dev, k):
    from graphneuralnetwork_amd.sampler import sample_neighbors
    adj = _adj(dev)
    rowptr = adj.rowptr.cpu().numpy()
    col = adj.col.cpu().numpy()
    deg = np.diff(rowptr)
    nodes = np.nonzero(deg > 0)[0]
    out = sample_neighbors(adj, torch.from_numpy(nodes), k, seed=3).cpu().numpy()
    again = sample_neighbors(adj, torch.from_numpy(nodes), k, seed=3).cpu().numpy()
    np.testing.assert_array_equal(out, again)
    for i, v in enumerate(nodes):
        nb = set(col[rowptr[v]:rowptr[v + 1]].tolist())
        assert set(out[i].tolist()) <= nb
        if deg[v] > k:
            assert len(set(out[i].tolist())) == k  # random.sample: distinct
    with pytest.raises(IndexError):
        iso = np.nonzero(deg == 0)[0]
        if iso.size == 0:
            raise IndexError("no isolated node in this graph")
        sample_neighbors(adj, torch.from_numpy(iso[:1]), k)


@pytest.mark.parametrize("k", [10, 25, 36])
def test_sample_is_uniform(dev, k):
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.sampler import sample_neighbors
    deg = 40
    rowptr = torch.tensor([0, deg], dtype=torch.int64, device=dev)
    col = torch.arange(deg, dtype=torch.int32, device=dev)
    g = CsrGraph(rowptr, col, torch.ones(deg, device=dev), 1, deg)
    nodes = torch.zeros(1, dtype=torch.int64, device=dev)
    counts = np.zeros(deg)
    for s in range(400):
        counts += np.bincount(sample_neighbors(g, nodes, k, seed=s).cpu().numpy()[0], minlength=deg)
    expected = 400 * k / deg
    chi2 = ((counts - expected) ** 2 / expected).sum()
    assert chi2 < 90  # 39 dof: p ~ 1e-5 threshold


def test_batch_maps_and_gathered_forward(dev):
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.sampler import sample_batch
    adj = _adj(dev)
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu().numpy()
    seeds = torch.from_numpy(np.nonzero(deg > 0)[0][:64]).to(dev)
    b = sample_batch(adj, seeds, fanouts=(25, 10), seed=1)
    assert torch.equal(b.frontier[b.center_map], seeds)
    assert b.frontier_nbrs.shape == (b.frontier.numel(), 10)
    assert b.neigh_map.shape == (64, 25)
    F = 32
    table = torch.randn(adj.n_rows, F, device=dev)
    net = GraphSAGE(2, F, 16, False, agg_func="MEAN", Unsupervised=False, class_size=3).to(dev).eval()
    with torch.no_grad():
        e1, c1 = net(*b.forward_args(table), None, None, None, None, None)
        pre = (table[b.frontier], [b.center_map], table[b.frontier_nbrs], [b.neigh_map])
        e2, c2 = net(*pre, None, None, None, None, None)
    torch.testing.assert_close(e1, e2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(c1, c2, rtol=1e-5, atol=1e-5)


def test_duplicate_nodes_and_layers_draw_independently(dev):
    """A node listed twice gets two independent neighbour lists, and batch s's layer 1
    does not replay batch s+1's layer 0 (the RNG was keyed by node and
    seed + layer)."""
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.sampler import sample_neighbors
    deg = 1000
    rowptr = torch.tensor([0, deg], dtype=torch.int64, device=dev)
    col = torch.arange(deg, dtype=torch.int32, device=dev)
    g = CsrGraph(rowptr, col, torch.ones(deg, device=dev), 1, deg)
    nodes = torch.zeros(4, dtype=torch.int64, device=dev)
    out = sample_neighbors(g, nodes, 10, seed=5).cpu().numpy()
    rows = {tuple(r) for r in out.tolist()}
    assert len(rows) == 4  # 10 of 1000: identical rows by chance have probability ~1e-30
    a = sample_neighbors(g, nodes[:1], 10, seed=5, layer=1).cpu().numpy()
    b = sample_neighbors(g, nodes[:1], 10, seed=6, layer=0).cpu().numpy()
    assert not np.array_equal(a, b)


@pytest.mark.parametrize("n_nodes,n_a,n_b", [(1, 1, 0), (31, 5, 40), (33, 33, 33),
                                             (100_000, 512, 12_800), (10_000_000, 8192, 204_800)])
def test_frontier_matches_unique_and_searchsorted(dev, n_nodes, n_a, n_b):
    """gnn_frontier_* (node bitmap + popcount scan) == torch.unique(cat) + searchsorted,
    bit for bit, incl. repeated ids, ids on word edges and a near-empty bitmap."""
    from graphneuralnetwork_amd.sampler import build_frontier
    g = torch.Generator(device=dev).manual_seed(n_nodes + n_a)
    a = torch.randint(0, n_nodes, (n_a,), device=dev, generator=g)
    b = torch.randint(0, n_nodes, (n_b,), device=dev, generator=g)
    if n_nodes > 64:
        b[:3] = torch.tensor([0, 31, n_nodes - 1], device=dev)
        a = torch.cat([a, a[:7]])  # duplicates inside one list
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    s1, rank = build_frontier(a, b.view(-1, 1) if n_b else b, n_nodes, err)
    ref = torch.unique(torch.cat([a, b]))
    assert torch.equal(s1, ref)
    assert torch.equal(rank(a), torch.searchsorted(ref, a))
    assert torch.equal(rank(b), torch.searchsorted(ref, b))


def test_batch_errors_and_frontier_out_of_range(dev):
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.sampler import build_frontier, sample_batch
    # node 2 has no neighbour: the reference's random.choices([]) IndexError
    rowptr = torch.tensor([0, 2, 3, 3], dtype=torch.int64, device=dev)
    col = torch.tensor([1, 0, 0], dtype=torch.int32, device=dev)
    g = CsrGraph(rowptr, col, torch.ones(3, device=dev), 3, 3)
    with pytest.raises(IndexError, match="empty sequence"):
        sample_batch(g, torch.tensor([0, 2], device=dev), (4, 2))
    with pytest.raises(IndexError, match="out of range"):
        sample_batch(g, torch.tensor([0, 7], device=dev), (4, 2))
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    with pytest.raises(IndexError, match="out of range"):
        build_frontier(torch.tensor([0, 5], device=dev), torch.tensor([1], device=dev), 3, err)
    b = sample_batch(g, torch.tensor([0, 1], device=dev), (4, 2), seed=3)
    assert torch.equal(b.frontier[b.center_map], torch.tensor([0, 1], device=dev))
    nb = b.frontier[b.neigh_map].cpu().numpy()   # every sampled id is a true neighbour
    assert set(nb[0]) <= {0, 1} and set(nb[1]) == {0}


@pytest.mark.parametrize("fanouts", [(5,), (25, 10), (10, 5, 3), (4, 3, 2, 2)])
@pytest.mark.parametrize("gcn", [False, True])
def test_multi_hop_batch(dev, fanouts, gcn):
    """L-hop frontier chain (get_layer_adj_nodes, GraphSAGE/data_utils.py:82-117, with a
    fanout per hop): S_{i+1} = sorted unique(S_i ++ sampled), the maps are positions in the
    next layer, every sampled id is a true neighbour; the L-layer forward on the maps equals
    the numpy oracle."""
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.sampler import sample_batch
    from oracle import gnn_oracle as O
    adj = _adj(dev)
    rowptr, col = adj.rowptr.cpu().numpy(), adj.col.cpu().numpy()
    deg = np.diff(rowptr)
    seeds = torch.from_numpy(np.nonzero(deg > 0)[0][:50]).to(dev)
    b = sample_batch(adj, seeds, fanouts, seed=4, gcn=gcn)
    L = len(fanouts)
    assert len(b.center_maps) == len(b.neigh_maps) == L - 1 and len(b.layer_sizes) == L
    layers = list(b.layers)
    assert torch.equal(layers[0], seeds) and torch.equal(layers[-1], b.frontier)
    for i in range(L - 1):  # forward order is reversed: layer i's maps are [L - 2 - i]
        cm, nm, nxt = b.center_maps[L - 2 - i], b.neigh_maps[L - 2 - i], layers[i + 1]
        assert torch.equal(nxt[cm], layers[i])
        k = fanouts[i] + (1 if gcn else 0)
        assert nm.shape == (layers[i].numel(), k)
        ids = nxt[nm].cpu().numpy()
        for r, v in enumerate(layers[i].cpu().numpy()):
            nbs = set(col[rowptr[v]:rowptr[v + 1]].tolist()) | ({int(v)} if gcn else set())
            assert set(ids[r].tolist()) <= nbs
        if gcn:
            assert (ids[:, -1] == layers[i].cpu().numpy()).all()
        assert torch.equal(nxt, torch.unique(torch.cat([layers[i], nxt[nm].view(-1)])))
    assert b.frontier_nbrs.shape == (b.frontier.numel(), fanouts[-1] + (1 if gcn else 0))
    assert b.sampled_edges == sum(layers[i].numel() * (fanouts[i] + gcn) for i in range(L))
    F, H = 16, 8
    table = torch.randn(adj.n_rows, F, device=dev)
    torch.manual_seed(1)
    net = GraphSAGE(L, F, H, False, agg_func="MEAN", Unsupervised=False, class_size=3).to(dev).eval()
    with torch.no_grad():
        emb, logits = net(*b.forward_args(table), None, None, None, None, None)
    tn = table.cpu().numpy()
    ref_emb, ref_logits = O.graphsage_forward(
        tn[b.frontier.cpu().numpy()], [m.cpu().numpy() for m in b.center_maps],
        tn[b.frontier_nbrs.cpu().numpy()], [m.cpu().numpy() for m in b.neigh_maps],
        [blk.weight.weight.detach().cpu().numpy() for blk in net.sage_blocks], "MEAN", False,
        (net.dense.weight.detach().cpu().numpy(), net.dense.bias.detach().cpu().numpy()))
    assert emb.shape == (seeds.numel(), H)
    np.testing.assert_allclose(emb.cpu().numpy(), ref_emb, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(logits.cpu().numpy(), ref_logits, rtol=1e-4, atol=1e-5)


def test_rank_after_rebuild_raises(dev):
    """a rank() of an older build_frontier must not read a newer workspace."""
    from graphneuralnetwork_amd.sampler import build_frontier
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    a = torch.tensor([3, 1, 4], device=dev)
    _, rank1 = build_frontier(a, a, 10, err)
    build_frontier(torch.tensor([2], device=dev), a, 10, err)
    with pytest.raises(RuntimeError, match="rebuilt"):
        rank1(a)


def test_fanout_validation(dev):
    from graphneuralnetwork_amd.sampler import sample_batch
    adj = _adj(dev)
    with pytest.raises(ValueError):
        sample_batch(adj, torch.tensor([0], device=dev), ())
    with pytest.raises(ValueError):
        sample_batch(adj, torch.tensor([0], device=dev), (3, 0))


def test_degree_ordered_dataset_forward(dev):
    """A batch sampled on the degree-ordered dataset (sampler.degree_ordered) is a batch of
    the original graph under perm: every sampled id is a true neighbour there, and the
    forward over (adj', table') equals the forward over the original table with the
    batch's ids mapped back, bit for bit."""
    from graphneuralnetwork_amd.graphsage import GraphSAGE, Gathered
    from graphneuralnetwork_amd.sampler import degree_ordered, sample_batch
    adj = _adj(dev, n=5000, e=60000, seed=3)
    F = 64
    table = torch.randn(adj.n_rows, F, device=dev)
    adj2, table2, o = degree_ordered(adj, table)
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu().numpy()
    seeds = torch.from_numpy(np.nonzero(deg > 0)[0][:300]).to(dev)
    b = sample_batch(adj2, o.inv[seeds], (25, 10), seed=2)
    perm = o.perm
    rowptr, col = adj.rowptr.cpu().numpy(), adj.col.cpu().numpy()
    fr = perm[b.frontier].cpu().numpy()
    nb = perm[b.frontier_nbrs].cpu().numpy()
    for i in range(0, fr.size, 97):
        assert set(nb[i].tolist()) <= set(col[rowptr[fr[i]]:rowptr[fr[i] + 1]].tolist())
    assert torch.equal(perm[b.frontier[b.center_map]], seeds)
    net = GraphSAGE(2, F, 32, False, agg_func="MEAN", Unsupervised=False, class_size=3).to(dev).eval()
    with torch.no_grad():
        e1, c1 = net(*b.forward_args(table2), None, None, None, None, None)
        nat = (Gathered(table, perm[b.frontier], True), b.forward_args(table2)[1],
               Gathered(table, perm[b.frontier_nbrs], True), b.forward_args(table2)[3])
        e2, c2 = net(*nat, None, None, None, None, None)
    assert torch.equal(e1, e2) and torch.equal(c1, c2)


@pytest.mark.parametrize("fanouts", [(5,), (25, 10), (10, 5, 3), (4, 3, 2, 2), (40, 20)])
@pytest.mark.parametrize("gcn", [False, True])
def test_fused_batch_equals_stepwise(dev, fanouts, gcn):
    """gnn_sample_layers (every hop on the device, one host read at the end) returns the same
    tensors as the hop-by-hop path, bit for bit: layers, neighbour lists and both maps, with
    repeated seeds; and raises the same errors."""
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.sampler import sample_batch, sample_batch_stepwise
    adj = _adj(dev, n=20000, e=150000, seed=3)
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu().numpy()
    cand = np.nonzero(deg > 0)[0]
    seeds = torch.from_numpy(np.concatenate([cand[:300], cand[:5]])).to(dev)
    a = sample_batch(adj, seeds, fanouts, seed=9, gcn=gcn)
    b = sample_batch_stepwise(adj, seeds, fanouts, seed=9, gcn=gcn)
    assert len(a.layers) == len(b.layers) == len(fanouts)
    for x, y in zip(a.layers, b.layers):
        assert torch.equal(x, y)
    assert torch.equal(a.frontier, b.frontier) and torch.equal(a.frontier_nbrs, b.frontier_nbrs)
    for xs, ys in ((a.center_maps, b.center_maps), (a.neigh_maps, b.neigh_maps)):
        assert len(xs) == len(ys)
        for x, y in zip(xs, ys):
            assert torch.equal(x, y)
    rowptr = torch.tensor([0, 2, 3, 3], dtype=torch.int64, device=dev)
    col = torch.tensor([1, 0, 0], dtype=torch.int32, device=dev)
    g = CsrGraph(rowptr, col, torch.ones(3, device=dev), 3, 3)
    for fn in (sample_batch, sample_batch_stepwise):
        with pytest.raises(IndexError, match="empty sequence"):
            fn(g, torch.tensor([0, 2], device=dev), fanouts, gcn=gcn)
        with pytest.raises(IndexError, match="out of range"):
            fn(g, torch.tensor([7, 0], device=dev), fanouts, gcn=gcn)


def test_fused_batch_leaves_workspace_clean(dev):
    """gnn_sample_layers' workspace contract: zero-filled before the first call, zero-filled
    flags again after every call (the scan clears what it reads), so back-to-back batches on
    different seeds and an erroring batch in between all give the step-by-step results."""
    from graphneuralnetwork_amd import sampler as S
    adj = _adj(dev, n=30000, e=200000, seed=5)
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu().numpy()
    cand = np.nonzero(deg > 0)[0]
    empty = np.nonzero(deg == 0)[0]
    n_words = (adj.n_rows + 31) // 32
    for it in range(4):
        seeds = torch.from_numpy(cand[it * 500:(it + 1) * 500]).to(dev)
        a = S.sample_batch(adj, seeds, (6, 4, 3), seed=it)
        b = S.sample_batch_stepwise(adj, seeds, (6, 4, 3), seed=it)
        assert torch.equal(a.frontier, b.frontier) and torch.equal(a.neigh_map, b.neigh_map)
        for x, y in zip(a.center_maps, b.center_maps):
            assert torch.equal(x, y)
        ws = S._SAMPLE_WS[(adj.device, adj.n_rows, torch.cuda.current_stream(dev).cuda_stream)]
        assert int(ws[:32 * n_words].count_nonzero()) == 0
        if empty.size and it == 1:
            with pytest.raises(IndexError):
                S.sample_batch(adj, torch.from_numpy(np.concatenate([cand[:10], empty[:1]])).to(dev),
                               (6, 4))
            assert int(ws[:32 * n_words].count_nonzero()) == 0


def test_fused_batch_full_size_cfg4(dev):
    """The cfg4 batch (8192 seeds, [25, 10]) on the 10M-node R-MAT adjacency: fused == stepwise."""
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import (sample_batch, sample_batch_stepwise,
                                                symmetric_adjacency)
    n = 10_000_000
    s, d = rmat_edges(n, 100_000_000, 0)
    adj = symmetric_adjacency(s, d, n, device=dev)
    del s, d
    gen = torch.Generator(device=dev).manual_seed(0)
    cand = torch.nonzero(adj.rowptr[1:] > adj.rowptr[:-1]).view(-1)
    seeds = cand[torch.randperm(cand.numel(), device=dev, generator=gen)[:8192]]
    a = sample_batch(adj, seeds, (25, 10), seed=0)
    b = sample_batch_stepwise(adj, seeds, (25, 10), seed=0)
    assert torch.equal(a.frontier, b.frontier) and torch.equal(a.frontier_nbrs, b.frontier_nbrs)
    assert torch.equal(a.center_map, b.center_map) and torch.equal(a.neigh_map, b.neigh_map)


def _draws_ref(rowptr, col, nodes, k, seed):
    """Python restatement of the device draw (sample_kernels.hpp): splitmix64 counter RNG keyed
    by (seed, position, draw), Lemire's multiply-shift, Floyd without replacement for deg > k,
    independent draws otherwise -- the exact picks every sampler kernel must produce."""
    M = (1 << 64) - 1

    def mix(z):
        z = (z + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    def below(pos, draw, n):
        r = mix(seed ^ mix((pos * 0x100000001B3 + draw) & M))
        return ((r >> 32) * n) >> 32

    out = np.full((len(nodes), k), -1, np.int64)
    for i, v in enumerate(nodes):
        b, deg = int(rowptr[v]), int(rowptr[v + 1] - rowptr[v])
        if deg == 0:
            continue
        if deg <= k:
            picks = [below(i, j, deg) for j in range(k)]
        else:
            picks = []
            for jj in range(k):
                j = deg - k + jj
                t = below(i, j, j + 1)
                picks.append(j if t in picks else t)
        out[i] = col[b + np.array(picks)]
    return out


@pytest.mark.parametrize("k", [1, 3, 10, 16, 17, 25, 32, 40, 64, 65])
def test_draws_match_restatement(dev, k):
    """Every sampler kernel (lane-parallel Floyd for k <= 64, thread-serial above) draws exactly
    the picks of the Python restatement, incl. nodes with deg <= k (choices) and hubs."""
    from graphneuralnetwork_amd.sampler import sample_neighbors, stream_seed
    adj = _adj(dev, n=3000, e=40000, seed=7)
    rowptr = adj.rowptr.cpu().numpy()
    col = adj.col.cpu().numpy()
    deg = np.diff(rowptr)
    nodes = np.concatenate([np.nonzero(deg > 0)[0][:300], np.argsort(-deg)[:8]])
    got = sample_neighbors(adj, torch.from_numpy(nodes).to(dev), k, seed=11, layer=1).cpu().numpy()
    want = _draws_ref(rowptr, col, nodes, k, stream_seed(11, 1))
    np.testing.assert_array_equal(got, want)


def test_degree_ordered_keeps_edge_values(dev):
    """sampler.degree_ordered re-sorts each row's neighbours; a weighted adjacency
    keeps every value on its own edge (the (row, col, val) triplets are P A P^T's)."""
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.sampler import degree_ordered
    adj = _adj(dev, n=2000, e=20000, seed=4)
    rowptr, col = adj.rowptr.cpu().numpy(), adj.col.cpu().numpy()
    rng = np.random.default_rng(0)
    val = rng.standard_normal(col.size).astype(np.float32)          # distinct per edge
    g = CsrGraph(adj.rowptr, adj.col, torch.from_numpy(val).to(dev), adj.n_rows, adj.n_cols)
    g2, _, o = degree_ordered(g)
    inv = o.inv.cpu().numpy()
    rows = np.repeat(np.arange(adj.n_rows), np.diff(rowptr))
    want = sorted(zip(inv[rows].tolist(), inv[col].tolist(), val.tolist()))
    rp2, c2, v2 = g2.rowptr.cpu().numpy(), g2.col.cpu().numpy(), g2.val.cpu().numpy()
    rows2 = np.repeat(np.arange(adj.n_rows), np.diff(rp2))
    assert sorted(zip(rows2.tolist(), c2.tolist(), v2.tolist())) == want
    for r in range(0, adj.n_rows, 97):                               # ascending neighbours
        assert np.all(np.diff(c2[rp2[r]:rp2[r + 1]]) > 0)


@pytest.mark.parametrize("fanouts,F,H", [((25, 10), 128, 128), ((10, 5, 3), 64, 128),
                                         ((25, 10), 32, 16)])
def test_pending_batch_forward_equals_synced(dev, fanouts, F, H):
    """sample_batch(..., sync=False): no host read between the sampler and the forward (the
    layer sizes stay on the device, the fused concat gather and MFMA GEMM read them); the
    embeddings and logits equal the synced batch's bit for bit, for the fused shapes
    (F = 128 / 64 -> H = 128) and for a shape the live path hands back to the host (F = 32),
    and sync() returns the synced batch's tensors."""
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.sampler import sample_batch
    adj = _adj(dev, n=40000, e=300000, seed=4)
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu().numpy()
    seeds = torch.from_numpy(np.nonzero(deg > 0)[0][:700]).to(dev)
    table = torch.randn(adj.n_rows, F, device=dev)
    net = GraphSAGE(len(fanouts), F, H, False, agg_func="MEAN", Unsupervised=False,
                    class_size=3).to(dev).eval()
    a = sample_batch(adj, seeds, fanouts, seed=11)
    p = sample_batch(adj, seeds, fanouts, seed=11, sync=False)
    assert p.pending and not a.pending
    assert p.frontier.numel() >= a.frontier.numel()  # the buffer at its capacity
    with torch.no_grad():
        e1, c1 = net(*a.forward_args(table), None, None, None, None, None)
        e2, c2 = net(*p.forward_args(table), None, None, None, None, None)
    assert torch.equal(e1, e2) and torch.equal(c1, c2)
    s = p.sync()
    assert not s.pending and s.layer_sizes == a.layer_sizes
    assert torch.equal(s.frontier, a.frontier) and torch.equal(s.frontier_nbrs, a.frontier_nbrs)
    for xs, ys in ((s.center_maps, a.center_maps), (s.neigh_maps, a.neigh_maps)):
        for x, y in zip(xs, ys):
            assert torch.equal(x, y)
    assert p.sampled_edges == a.sampled_edges
    # the fused MAX / MAXPOOL layers run on the device sizes too; the non-fused path
    # (autograd) reads the sizes back and slices: same results as the synced batch
    for agg, grad in (("MAX", False), ("MAXPOOL", False), ("MEAN", True)):
        net.agg_func = agg
        with torch.set_grad_enabled(grad):
            e3, _ = net(*a.forward_args(table), None, None, None, None, None)
            e4, _ = net(*sample_batch(adj, seeds, fanouts, seed=11, sync=False).forward_args(table),
                        None, None, None, None, None)
        assert torch.equal(e3, e4)


def test_pending_batch_errors_raise_at_check(dev):
    """A pending batch with a sampler error (a seed without neighbours, an id out of range):
    the forward runs on the flawed lists without faulting (its gathers are range-checked) and
    check() raises the error sample_batch(..., sync=True) raises."""
    from graphneuralnetwork_amd.graph import CsrGraph
    from graphneuralnetwork_amd.graphsage import GraphSAGE
    from graphneuralnetwork_amd.sampler import sample_batch
    rowptr = torch.tensor([0, 2, 3, 3], dtype=torch.int64, device=dev)
    col = torch.tensor([1, 0, 0], dtype=torch.int32, device=dev)
    g = CsrGraph(rowptr, col, torch.ones(3, device=dev), 3, 3)
    table = torch.randn(3, 64, device=dev)
    net = GraphSAGE(2, 64, 128, False, agg_func="MEAN", Unsupervised=False,
                    class_size=3).to(dev).eval()
    for seeds, match in (([0, 2], "empty sequence"), ([7, 0], "out of range")):
        p = sample_batch(g, torch.tensor(seeds, device=dev), (4, 2), sync=False)
        with torch.no_grad():
            net(*p.forward_args(table), None, None, None, None, None)
        with pytest.raises(IndexError, match=match):
            p.check()
    torch.cuda.synchronize()
    ok = sample_batch(g, torch.tensor([0, 1], device=dev), (4, 2), sync=False)
    ok.check()


@pytest.mark.gpu
def test_pending_batch_synced_off_its_stream(dev):
    """a batch sampled pending under a side stream and synced on another reads its
    sizes on the sampler's stream (the copy waits for the scan), and each stream keeps its own
    workspace. Equal to the batch sampled and synced on the default stream."""
    from graphneuralnetwork_amd import sampler as S
    adj = _adj(dev, n=40000, e=300000, seed=4)
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu().numpy()
    seeds = torch.from_numpy(np.nonzero(deg > 0)[0][:700]).to(dev)
    a = S.sample_batch(adj, seeds, (25, 10), seed=5)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        torch.cuda._sleep(2_000_000)  # keep the side stream busy ahead of the sampler
        p = S.sample_batch(adj, seeds, (25, 10), seed=5, sync=False)
    s = p.sync()  # on the default stream: must still wait for the side stream's kernels
    assert s.layer_sizes == a.layer_sizes
    torch.cuda.current_stream(dev).wait_stream(side)
    assert torch.equal(s.frontier, a.frontier) and torch.equal(s.neigh_map, a.neigh_map)
    keys = [k for k in S._SAMPLE_WS if k[1] == adj.n_rows]
    assert len({k[2] for k in keys}) == 2
