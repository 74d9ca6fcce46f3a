"""Generate the golden vectors in tests/golden/ by running the REFERENCE code.

Run in the build container only (needs /root/reference, read-only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

For each model family a fresh subprocess puts the reference directory on
sys.path, imports the reference modules (no bytecode is written), builds small
seeded synthetic inputs in the reference's own formats, runs the reference
forward passes on CPU and stores inputs + outputs as compressed .npz
fixtures.  Nothing from the reference is copied: only data is written.
Parameters are drawn from a small dyadic grid (k/64) so the fixtures compress
well and are exactly representable in fp32.
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference")


def _q(rng, shape, scale=64, lim=64):
    """Dyadic random values k/scale, k in [-lim, lim]."""
    return (rng.integers(-lim, lim + 1, size=shape) / scale).astype(np.float32)


def _set_params(module, rng, scale=64, lim=48):
    import torch
    with torch.no_grad():
        for p in module.parameters():
            p.copy_(torch.from_numpy(_q(rng, tuple(p.shape), scale, lim)))


# ----------------------------------------------------------------------- GCN
def _write_cora(d: Path, rng, n=2708, n_feat=1433, n_cls=7, n_cites=5429):
    ids = rng.choice(np.arange(10_000, 10_000 + 20 * n), size=n, replace=False)
    labels = [f"Class_{c}" for c in rng.integers(0, n_cls, size=n)]
    with open(d / "cora.content", "w") as f:
        for i in range(n):
            row = np.zeros(n_feat, dtype=np.int64)
            row[rng.choice(n_feat, size=int(rng.integers(5, 30)), replace=False)] = 1
            f.write(f"{ids[i]}\t" + "\t".join(map(str, row)) + f"\t{labels[i]}\n")
    # power-law-ish cites: a few hubs, duplicates allowed, no self cites needed
    w = 1.0 / np.arange(1, n + 1) ** 0.8
    w /= w.sum()
    src = rng.choice(n, size=n_cites, p=w)
    dst = rng.integers(0, n, size=n_cites)
    with open(d / "cora.cites", "w") as f:
        for s, t in zip(src, dst):
            f.write(f"{ids[s]}\t{ids[t]}\n")
    return ids, src, dst


def part_gcn():
    sys.path.insert(0, str(REF / "GCN"))
    import torch
    import data_utils as du  # reference GCN/data_utils.py
    import scipy.sparse as sp
    from GCN import GCN_Model, Graph_conv_layer  # reference GCN/GCN.py

    torch.manual_seed(0)
    rng = np.random.default_rng(0)
    out = {}
    # -- cfg1: Cora-format synthetic through the full reference loader + model
    with tempfile.TemporaryDirectory() as td:
        d = Path(td)
        ids, src, dst = _write_cora(d, rng)
        adj, features, labels, *_ = du.load_cora(data_dir=str(d) + "/", dataset="cora")
    model = GCN_Model(features.shape[1], num_hidden=128, num_classes=7, num_layers=2, dropout=0.5)
    _set_params(model, rng, lim=16)
    model.eval()
    with torch.no_grad():
        logits = model(features, adj)
    sd = model.state_dict()
    fnz = features.nonzero().numpy()
    idx = adj._indices().numpy()
    np.savez_compressed(
        HERE / "gcn_cora.npz",
        edges=np.stack([src, dst], 1).astype(np.int32),  # node indices (file order)
        adj_row=idx[0].astype(np.int32), adj_col=idx[1].astype(np.int32),
        adj_val=adj._values().numpy(), n=np.int64(features.shape[0]),
        feat_row=fnz[:, 0].astype(np.int32), feat_col=fnz[:, 1].astype(np.int16),
        feat_val=features[fnz[:, 0], fnz[:, 1]].numpy(), n_feat=np.int64(features.shape[1]),
        w0=sd["gcn_blocks.gcn0.dense.weight"].numpy(), b0=sd["gcn_blocks.gcn0.bias"].numpy(),
        w1=sd["gcn_blocks.gcn1.dense.weight"].numpy(), b1=sd["gcn_blocks.gcn1.bias"].numpy(),
        logits=logits.numpy(), state_keys=np.array(list(sd.keys())))
    print("gcn_cora.npz", logits.shape)

    # -- SpMM graphs through the reference preprocessing + Graph_conv_layer (W = I)
    def ref_adj(n, s, t):
        feats = np.zeros((n, 3), dtype=object)
        feats[:, 0] = np.arange(n).astype(str)
        feats[:, 1] = "1"
        feats[:, 2] = "c"
        node2idx = {i: i for i in range(n)}
        edges_un = np.stack([s, t], 1).astype(np.int32)
        _, _, a = du.preprocess_data(feats, edges_un, node2idx)
        a = du.normalize_adj(a + sp.eye(a.shape[0]))
        return du.sparse_mx_to_torch_sparse_tensor(a)

    cases = []
    # g1: duplicates, a 600-edge hub, isolated nodes
    n = 1000
    s = rng.integers(0, 900, size=4000)
    t = rng.integers(0, 900, size=4000)
    s = np.concatenate([s, np.zeros(600, np.int64), s[:300]])      # hub 0 + 300 duplicates
    t = np.concatenate([t, rng.choice(900, 600, replace=False), t[:300]])
    cases.append(("g1", n, s, t, [7, 64]))
    # g2: RMAT (survey recipe, scale 12) folded onto 3000 nodes
    scale, ne = 12, 24000
    r2 = np.random.default_rng(2)
    rs = np.zeros(ne, np.int64)
    cs = np.zeros(ne, np.int64)
    for b in range(scale):
        u = r2.random(ne)
        v = r2.random(ne)
        rb = u > 0.57 + 0.19
        cb = np.where(rb, v < 0.05 / (0.19 + 0.05), v < 0.19 / (0.57 + 0.19))
        rs |= rb.astype(np.int64) << b
        cs |= cb.astype(np.int64) << b
    cases.append(("g2", 3000, rs % 3000, cs % 3000, [128, 256]))
    # g3: tiny, every node isolated except a chain
    cases.append(("g3", 257, np.arange(0, 100), np.arange(1, 101), [1, 5, 33]))
    arrays = {}
    for name, n, s, t, feats in cases:
        A = ref_adj(n, s, t)
        i = A._indices().numpy()
        arrays[f"{name}_n"] = np.int64(n)
        arrays[f"{name}_edges"] = np.stack([s, t], 1).astype(np.int32)
        arrays[f"{name}_row"] = i[0].astype(np.int32)
        arrays[f"{name}_col"] = i[1].astype(np.int32)
        arrays[f"{name}_val"] = A._values().numpy()
        deg = np.bincount(i[0], minlength=n)
        check = np.unique(np.concatenate([rng.choice(n, size=min(n, 192), replace=False),
                                          np.argsort(-deg)[:8], np.nonzero(deg <= 1)[0][:8]]))
        for F in feats:
            layer = Graph_conv_layer(F, F)
            with torch.no_grad():
                layer.dense.weight.copy_(torch.eye(F))
                layer.bias.copy_(torch.from_numpy(_q(rng, (F,), 16, 16)))
            X = (rng.integers(-16, 17, size=(n, F)) / 8).astype(np.float32)
            with torch.no_grad():
                Y = layer(torch.from_numpy(X), A).numpy()
            arrays[f"{name}_F{F}_xq"] = (X * 8).astype(np.int8)
            arrays[f"{name}_F{F}_bias"] = layer.bias.detach().numpy()
            arrays[f"{name}_F{F}_rows"] = check.astype(np.int32)
            arrays[f"{name}_F{F}_y"] = Y[check]
        print(name, n, A._nnz(), feats)
    arrays["cases"] = np.array([c[0] for c in cases])
    arrays["feats"] = np.array([",".join(map(str, c[4])) for c in cases])
    np.savez_compressed(HERE / "gcn_spmm.npz", **arrays)


# ----------------------------------------------------------------------- GAT
def part_gat():
    import importlib.util
    import torch
    spec = importlib.util.spec_from_file_location("ref_gat_layers", REF / "GAT/models/layers.py")
    L = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(L)
    torch.manual_seed(0)
    rng = np.random.default_rng(3)
    N, Fin, H, Fh, C, alpha = 512, 64, 8, 8, 7, 0.2
    # adjacency: symmetric, self loops, positive normalised-looking values
    s = rng.integers(0, N, 3000)
    t = rng.integers(0, N, 3000)
    A = np.zeros((N, N), np.float32)
    A[s, t] = 1
    A[t, s] = 1
    A[np.arange(N), np.arange(N)] = 1
    A[5, :] = 0
    A[5, 5] = 1                            # a degree-1 row
    A[7, :50] = 1                          # a hub-ish row
    A = A * (rng.integers(1, 5, (N, N)) / 4).astype(np.float32)
    h = _q(rng, (N, Fin), 32, 32)
    adj = torch.from_numpy(A)
    ht = torch.from_numpy(h)
    out = {"adj_row": None}
    for kind, cls in (("dense", L.GraphAttentionLayer), ("sparse", L.SpGraphAttentionLayer)):
        heads = [cls(Fin, Fh, dropout=0.6, alpha=alpha, concat=True) for _ in range(H)]
        out_att = cls(Fh * H, C, dropout=0.6, alpha=alpha, concat=False)
        for m in heads + [out_att]:
            _set_params(m, rng, 64, 40)
            m.eval()
        with torch.no_grad():
            head0 = heads[0](ht, adj)
            x = torch.cat([m(ht, adj) for m in heads], dim=1)       # GAT/models/GAT.py:16
            logits = torch.nn.functional.elu(out_att(x, adj))       # GAT/models/GAT.py:18
        out[f"{kind}_W"] = np.stack([m.W.detach().numpy() for m in heads])
        out[f"{kind}_a"] = np.stack([m.a.detach().numpy().reshape(-1) for m in heads])
        out[f"{kind}_outW"] = out_att.W.detach().numpy()
        out[f"{kind}_outa"] = out_att.a.detach().numpy().reshape(-1)
        out[f"{kind}_head0"] = head0.numpy()
        out[f"{kind}_concat"] = x.numpy()
        out[f"{kind}_logits"] = logits.numpy()
        print("gat", kind, logits.shape)
    # dense-vs-nonzero edge sets: a matrix with negative entries, one head each
    An = A.copy()
    An[np.arange(0, N, 3), np.arange(1, N, 3)[: len(range(0, N, 3))]] = -0.5
    adjn = torch.from_numpy(An)
    dl = L.GraphAttentionLayer(Fin, Fh, dropout=0.0, alpha=alpha, concat=True)
    sl = L.SpGraphAttentionLayer(Fin, Fh, dropout=0.0, alpha=alpha, concat=True)
    for m in (dl, sl):
        _set_params(m, rng, 64, 40)
        m.eval()
    with torch.no_grad():
        out["neg_dense_out"] = dl(ht, adjn).numpy()
        out["neg_sparse_out"] = sl(ht, adjn).numpy()
    out["neg_dense_W"], out["neg_dense_a"] = dl.W.detach().numpy(), dl.a.detach().numpy().reshape(-1)
    out["neg_sparse_W"], out["neg_sparse_a"] = sl.W.detach().numpy(), sl.a.detach().numpy().reshape(-1)
    # isolated row: dense gives a uniform average, sparse raises (NaN assert)
    Ai = A.copy()
    Ai[9, :] = 0
    with torch.no_grad():
        out["iso_dense_out"] = dl(ht, torch.from_numpy(Ai)).numpy()
        try:
            sl(ht, torch.from_numpy(Ai))
            out["iso_sparse_raises"] = np.int64(0)
        except AssertionError:
            out["iso_sparse_raises"] = np.int64(1)
    nz = np.nonzero(A)
    out.pop("adj_row")
    out.update(adj_row=nz[0].astype(np.int32), adj_col=nz[1].astype(np.int32), adj_val=A[nz],
               neg_row=np.nonzero(An)[0].astype(np.int32), neg_col=np.nonzero(An)[1].astype(np.int32),
               neg_val=An[np.nonzero(An)], h=h, n=np.int64(N), alpha=np.float64(alpha),
               iso_row=np.int64(9))
    np.savez_compressed(HERE / "gat.npz", **out)


# ------------------------------------------------------------- GAT gradients
def part_gatgrad():
    """Gradients of the 8-head attention block (GAT/models/GAT.py:16: the heads of
    layers.py:22-37 / :94-131 concatenated) under autograd -- the reference's own backward,
    SpecialSpmmFunction.backward (layers.py:54-64) for the sparse heads -- for the loss
    sum(block(h, adj) * gy): pins the float64 C restatement (oracle_gat_block_grad) that the
    full-size training test checks the HIP backward against. Dropout 0 (torch's RNG stream is
    not the HIP kernels' hash; the hash is restated and checked separately)."""
    import importlib.util
    import torch
    spec = importlib.util.spec_from_file_location("ref_gat_layers", REF / "GAT/models/layers.py")
    L = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(L)
    torch.manual_seed(0)
    rng = np.random.default_rng(11)
    N, Fin, H, Fh, alpha = 384, 64, 8, 8, 0.2
    s = rng.integers(0, N, 2500)
    t = rng.integers(0, N, 2500)
    A = np.zeros((N, N), np.float32)
    A[s, t] = 1
    A[t, s] = 1
    A[np.arange(N), np.arange(N)] = 1
    A[11, :] = 0
    A[11, 11] = 1                          # a degree-1 row
    A[:60, 3] = 1                          # a hub column
    A[3, :60] = 1
    h = _q(rng, (N, Fin), 32, 32)
    gy = _q(rng, (N, H * Fh), 16, 16)
    out = {"adj_row": np.nonzero(A)[0].astype(np.int32), "adj_col": np.nonzero(A)[1].astype(np.int32),
           "h": h, "gy": gy, "n": np.int64(N), "alpha": np.float64(alpha), "heads": np.int64(H),
           "fh": np.int64(Fh)}
    for kind, cls in (("dense", L.GraphAttentionLayer), ("sparse", L.SpGraphAttentionLayer)):
        heads = [cls(Fin, Fh, dropout=0.0, alpha=alpha, concat=True) for _ in range(H)]
        for m in heads:
            _set_params(m, rng, 64, 40)
            m.train()
        ht = torch.from_numpy(h).requires_grad_(True)
        x = torch.cat([m(ht, torch.from_numpy(A)) for m in heads], dim=1)   # GAT/models/GAT.py:16
        (x * torch.from_numpy(gy)).sum().backward()
        out[f"{kind}_W"] = np.stack([m.W.detach().numpy() for m in heads])
        out[f"{kind}_a"] = np.stack([m.a.detach().numpy().reshape(-1) for m in heads])
        out[f"{kind}_out"] = x.detach().numpy()
        out[f"{kind}_dW"] = np.stack([m.W.grad.numpy() for m in heads])
        out[f"{kind}_da"] = np.stack([m.a.grad.numpy().reshape(-1) for m in heads])
        out[f"{kind}_dh"] = ht.grad.numpy()
        print("gatgrad", kind, x.shape)
    np.savez_compressed(HERE / "gatgrad.npz", **out)


# ----------------------------------------------------------------- GraphSAGE
def part_sage():
    sys.path.insert(0, str(REF / "GraphSAGE"))
    import random
    from collections import defaultdict
    import torch
    import data_utils as du  # reference GraphSAGE/data_utils.py
    from GraphSAGE import GraphSAGE  # reference GraphSAGE/GraphSAGE.py
    from graph_utils import Aggregator  # reference GraphSAGE/graph_utils.py

    random.seed(0)
    torch.manual_seed(0)
    rng = np.random.default_rng(5)
    N, F, Hd, K, B = 200, 32, 16, 5, 16
    adj_lists = defaultdict(set)
    for i in range(N):  # ring (deg >= 2) + random chords + a hub
        adj_lists[i].add((i + 1) % N)
        adj_lists[(i + 1) % N].add(i)
    for s, t in rng.integers(0, N, (300, 2)):
        if s != t:
            adj_lists[int(s)].add(int(t))
            adj_lists[int(t)].add(int(s))
    for t in range(1, 60):
        adj_lists[0].add(t)
        adj_lists[t].add(0)
    feat = _q(rng, (N, F), 16, 32)
    feat_list = feat.tolist()
    out = {"feat": feat}
    batch_nodes = [int(v) for v in rng.choice(N, B, replace=False)]
    labels = [int(v) for v in rng.integers(0, 3, B)]
    for tag, agg, gcn in (("mean", "MEAN", False), ("max", "MAX", False), ("gcn", "MEAN", True)):
        col = du.collate_fn(adj_lists, feat_list, 2, K, gcn, False)
        X, y = col(list(zip(batch_nodes, labels)))
        net = GraphSAGE(2, F, Hd, gcn, agg_func=agg, Unsupervised=False, class_size=3)
        _set_params(net, rng, 64, 24)
        net.eval()
        with torch.no_grad():
            emb, logits = net(*X, None, None, None, None, None)
            agg0 = Aggregator(X[2], agg)
        out[f"{tag}_center_feats"] = X[0].numpy()
        out[f"{tag}_nodes_map"] = X[1].numpy()
        out[f"{tag}_neigh_feats"] = X[2].numpy()
        out[f"{tag}_neigh_map"] = X[3].numpy()
        out[f"{tag}_agg0"] = agg0.numpy()
        for k, v in net.state_dict().items():
            out[f"{tag}_sd_{k}"] = v.numpy()
        out[f"{tag}_emb"] = emb.numpy()
        out[f"{tag}_logits"] = logits.numpy()
        print("sage", tag, emb.shape, X[2].shape)
    # unsupervised branch (GraphSAGE.py:54-61): contexts + negatives
    col = du.collate_fn(adj_lists, feat_list, 2, K, False, True)
    data = []
    for v in batch_nodes[:6]:
        ctx = random.choices(list(adj_lists[v]), k=2)
        neg = [int(x) for x in rng.choice(N, 3, replace=False)]
        data.append((v, ctx, neg))
    X, y = col(data)
    net = GraphSAGE(2, F, Hd, False, agg_func="MEAN", Unsupervised=True)
    _set_params(net, rng, 64, 24)
    net.eval()
    with torch.no_grad():
        emb, scores = net(*X, y.shape)
    for i, t in enumerate(X):
        out[f"unsup_X{i}"] = t.numpy()
    out["unsup_shape"] = np.array(y.shape)
    for k, v in net.state_dict().items():
        out[f"unsup_sd_{k}"] = v.numpy()
    out["unsup_emb"] = emb.numpy()
    out["unsup_scores"] = scores.numpy()
    np.savez_compressed(HERE / "sage.npz", **out)
    print("sage unsup", emb.shape, scores.shape)


# ----------------------------------------------------------------------- HAN
def part_han():
    """HAN node-level attention (GATConv per metapath) + semantic attention, 2 layers."""
    sys.path.insert(0, str(REF / "HAN"))
    import torch
    from models import HANModel                       # HAN/models/__init__.py
    rng = np.random.default_rng(11)
    torch.manual_seed(0)
    N, M, Fin, hid, C = 300, 3, 32, 8, 3
    heads = [4, 2]
    gs = []
    for _ in range(M):
        A = np.zeros((N, N), np.float32)
        s, t = rng.integers(0, N, 1500), rng.integers(0, N, 1500)
        A[s, t] = 1
        A[t, s] = 1
        A[np.arange(N), np.arange(N)] = 1             # metapath graphs keep self loops
        gs.append(A)
    h = _q(rng, (N, Fin), 32, 32)
    net = HANModel(M, Fin, hid, C, heads, dropout=0.6)
    _set_params(net, rng, 64, 40)
    net.eval()
    with torch.no_grad():
        gt = [torch.from_numpy(a) for a in gs]
        layer0 = net.layers[0](gt, torch.from_numpy(h))
        logits = net(gt, torch.from_numpy(h))
    out = {"h": h, "heads": np.array(heads), "layer0": layer0.numpy(), "logits": logits.numpy()}
    for i, a in enumerate(gs):
        nz = np.nonzero(a)
        out[f"g{i}_row"], out[f"g{i}_col"] = nz[0].astype(np.int32), nz[1].astype(np.int32)
    for k, v in net.state_dict().items():
        out[f"sd_{k}"] = v.numpy()
    out["dims"] = np.array([N, M, Fin, hid, C])
    np.savez_compressed(HERE / "han.npz", **out)
    print("han", logits.shape, len(net.state_dict()))


# ------------------------------------------------------- GraphSAGE_Pytorch
def part_sagepy():
    """GraphSAGE_Pytorch GraphSage over pre-sampled hop features + SageGCN variants."""
    sys.path.insert(0, str(REF / "GraphSAGE_Pytorch"))
    import torch
    from models import GraphSage, SageGCN             # GraphSAGE_Pytorch/models/__init__.py
    from models.Aggregator import NeighborAggregator
    rng = np.random.default_rng(12)
    torch.manual_seed(0)
    Fin, hidden, nbrs, B = 32, [16, 5], [10, 5], 20
    feats = [_q(rng, (B, Fin), 32, 32), _q(rng, (B * nbrs[0], Fin), 32, 32),
             _q(rng, (B * nbrs[0] * nbrs[1], Fin), 32, 32)]
    net = GraphSage(Fin, hidden, nbrs)
    _set_params(net, rng, 64, 40)
    with torch.no_grad():
        y = net([torch.from_numpy(f) for f in feats])
    out = {f"X{i}": f for i, f in enumerate(feats)}
    out["y"] = y.numpy()
    for k, v in net.state_dict().items():
        out[f"sd_{k}"] = v.numpy()
    # SageGCN with 'sum' neighbours + 'concat' hidden, and a biased 'mean' aggregator
    src, nb = torch.from_numpy(feats[0]), torch.from_numpy(feats[1]).view(B, nbrs[0], Fin)
    layer = SageGCN(Fin, 12, aggr_neighbor_method="sum", aggr_hidden_method="concat")
    agg = NeighborAggregator(Fin, 7, use_bias=True, aggr_method="mean")
    for m in (layer, agg):
        _set_params(m, rng, 64, 40)
    with torch.no_grad():
        out["sumcat_y"] = layer(src, nb).numpy()
        out["biasmean_y"] = agg(nb).numpy()
    for k, v in layer.state_dict().items():
        out[f"sumcat_sd_{k}"] = v.numpy()
    for k, v in agg.state_dict().items():
        out[f"biasmean_sd_{k}"] = v.numpy()
    try:                                              # 'max' gets a namedtuple -> matmul fails
        NeighborAggregator(Fin, 7, aggr_method="max")(nb)
        out["max_raises"] = np.int64(0)
    except TypeError:
        out["max_raises"] = np.int64(1)
    out["dims"] = np.array([Fin, B] + hidden + nbrs)
    np.savez_compressed(HERE / "sagepy.npz", **out)
    print("sagepy", y.shape)


# ------------------------------------------------------- GraphSAGE sampler (index maps)
def part_pysampler():
    """The reference's host sampler (get_layer_adj_nodes, GraphSAGE/data_utils.py:82-124)
    under a seeded global ``random``: pins the CPython-exact native sampler bit for bit.
    adj_lists is built exactly as read_pubmed_data does (data_utils.py:29-37) from a pair
    stream that is stored, so the native construction is pinned too."""
    sys.path.insert(0, str(REF / "GraphSAGE"))
    import random
    from collections import defaultdict
    import data_utils as du  # reference GraphSAGE/data_utils.py

    rng = np.random.default_rng(11)
    out = {}
    graphs = {}
    for name, N, E, hub in (("small", 300, 700, 90), ("mid", 20000, 90000, 700)):
        ring = np.stack([np.arange(N), (np.arange(N) + 1) % N], 1)  # every node has deg >= 2
        rnd = rng.integers(0, N, (E, 2))
        rnd[::97, 1] = rnd[::97, 0]                                   # self pairs
        hubs = np.stack([np.zeros(hub, np.int64), rng.integers(1, N, hub)], 1)
        pairs = np.concatenate([ring, rnd, hubs]).astype(np.int64)
        perm = rng.permutation(len(pairs))
        pairs = pairs[perm]
        adj = defaultdict(set)
        for a, b in pairs.tolist():
            adj[a].add(b)
            adj[b].add(a)
        order = [list(adj[v]) for v in range(N)]
        out[f"{name}_pairs"] = pairs
        out[f"{name}_n"] = np.int64(N)
        out[f"{name}_adj_ptr"] = np.cumsum([0] + [len(o) for o in order]).astype(np.int64)
        out[f"{name}_adj_nbr"] = np.asarray([u for o in order for u in o], np.int64)
        graphs[name] = adj
    cases = [("small", 20, 2, 5, False, 1), ("small", 20, 2, 5, True, 2),
             ("small", 10, 3, 4, False, 3), ("small", 12, 1, 7, False, 4),
             ("small", 16, 2, 30, False, 5), ("small", 8, 3, 3, True, 6),
             ("mid", 256, 2, 10, False, 7), ("mid", 128, 2, 25, False, 8),
             ("mid", 200, 2, 8, True, 9)]
    for c, (g, B, L, K, gcn, seed) in enumerate(cases):
        random.seed(seed)
        nodes = [int(v) for v in rng.choice(int(out[f"{g}_n"]), B, replace=False)]
        if c == 3:
            nodes[3] = nodes[1]  # a repeated batch node (dict position: last one wins)
        state0 = np.asarray(random.getstate()[1], np.uint32)
        neigh, center = du.get_layer_adj_nodes(nodes, graphs[g], L, K, gcn)
        out[f"case{c}_meta"] = np.array([["small", "mid"].index(g), L, K, int(gcn), seed])
        out[f"case{c}_nodes"] = np.asarray(nodes, np.int64)
        out[f"case{c}_state0"] = state0
        out[f"case{c}_neigh"] = np.asarray(neigh, np.int64)
        out[f"case{c}_center"] = np.asarray(center, np.int64)
        out[f"case{c}_state1"] = np.asarray(random.getstate()[1], np.uint32)
        print("pysampler case", c, out[f"case{c}_neigh"].shape)
    # a node without neighbours: random.choices on [] -> IndexError
    adj = defaultdict(set, {0: {1}, 1: {0}})
    random.seed(0)
    try:
        du.get_layer_adj_nodes([0, 5], adj, 1, 3, False)
        out["empty_raises"] = np.int64(0)
    except IndexError:
        out["empty_raises"] = np.int64(1)
    out["empty_state1"] = np.asarray(random.getstate()[1], np.uint32)
    np.savez_compressed(HERE / "pysampler.npz", **out)


def part_features():
    """GCN/data_utils.py normalize_features (row normalisation of the feature matrix) on
    real-valued float32 matrices, through the reference's own function and load_cora's
    torch.Tensor(features.toarray()) (GCN/data_utils.py:81-83)."""
    sys.path.insert(0, str(REF / "GCN"))
    import torch
    import data_utils as du  # reference GCN/data_utils.py
    import scipy.sparse as sp

    rng = np.random.default_rng(5)
    mats = {}
    # 1: Cora-like shape, ~2 % density, varied magnitudes; 2: long rows (pairwise splits
    # past 128 and 256 stored values), zero rows, rows whose sum is exactly 0 or negative
    n, f = 600, 1433
    x = np.where(rng.random((n, f)) < 0.02,
                 rng.standard_normal((n, f)) * rng.choice([1e-3, 1.0, 1e3], size=(n, 1)), 0)
    x[::50] = 0
    mats["a"] = x.astype(np.float32)
    n, f = 64, 1100
    y = np.zeros((n, f), np.float32)
    for i in range(n):
        k = int(rng.integers(0, f))
        cols = rng.choice(f, size=k, replace=False)
        y[i, cols] = rng.standard_normal(k).astype(np.float32) * 10
    y[3] = 0
    y[4] = 0
    y[4, :3] = (1.5, -1.5, 0.0)   # sum exactly 0 -> inf -> 0 (and 0 x -1.5)
    y[5] = -np.abs(y[5])          # negative sum
    mats["b"] = y
    out = {}
    for k, m in mats.items():
        norm = du.normalize_features(sp.csr_matrix(m, dtype=np.float32))
        out[f"x_{k}"] = m
        out[f"y_{k}"] = torch.Tensor(norm.toarray()).numpy()
    np.savez_compressed(HERE / "gcn_features.npz", **out)
    print("gcn_features.npz", {k: v.shape for k, v in out.items()})


PARTS = {"gcn": part_gcn, "features": part_features, "gat": part_gat, "gatgrad": part_gatgrad,
         "sage": part_sage, "han": part_han,
         "sagepy": part_sagepy, "pysampler": part_pysampler}

if __name__ == "__main__":
    sys.dont_write_bytecode = True
    if len(sys.argv) > 2 and sys.argv[1] == "--part":
        PARTS[sys.argv[2]]()
        sys.exit(0)
    if not REF.exists():
        sys.exit("the reference is not mounted at /root/reference: fixtures cannot be regenerated")
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", PYTHONHASHSEED="0")
    for p in (sys.argv[1:] or list(PARTS)):
        subprocess.run([sys.executable, __file__, "--part", p], check=True, env=env,
                       cwd=tempfile.gettempdir())
