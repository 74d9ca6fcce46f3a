"""Pin the CPU oracle against the reference's own outputs (golden vectors).

The fixtures in tests/golden/ were produced by running the reference code
(tests/golden/make_golden.py).  These tests need no GPU.
"""
import numpy as np
import pytest

from oracle import c_oracle
from oracle import gnn_oracle as O

RTOL = 1e-4


def close(a, b, rtol=RTOL, atol_frac=1e-4):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(1.0, float(np.abs(b).max())) if b.size else 1.0
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol_frac * scale)


def _csr_from_ref(row, col, val, n):
    return O.coo_to_csr(row.astype(np.int64), col, val, n)


# ------------------------------------------------------------------ GCN
def test_gcn_adjacency_pipeline_matches_reference(golden):
    """C3 -> +I -> C2 -> fp32 (GCN/data_utils.py:27-36,54-70): structure bit-exact, values bit-exact fp32."""
    g = golden("gcn_cora")
    n = int(g["n"])
    rowptr, col, val = O.gcn_adjacency(g["edges"][:, 0], g["edges"][:, 1], n)
    rr, rc, rv = _csr_from_ref(g["adj_row"], g["adj_col"], g["adj_val"], n)
    np.testing.assert_array_equal(rowptr, rr)
    # per-row column order may differ (reference is CSC order); compare sorted rows
    key_o = np.lexsort((col, np.repeat(np.arange(n), np.diff(rowptr))))
    key_r = np.lexsort((rc, np.repeat(np.arange(n), np.diff(rr))))
    np.testing.assert_array_equal(col[key_o], rc[key_r])
    np.testing.assert_array_equal(val[key_o], rv[key_r])


def test_normalize_features_matches_reference(golden):
    """C5 normalize_features (GCN/data_utils.py:39-51, then torch.Tensor(.toarray()) at
    :81-83): bit-exact on real-valued matrices (pairwise row sums past 128 and 256 values,
    zero rows, an exactly-zero and a negative row sum) and on the Cora fixture's binary
    features."""
    g = golden("gcn_features")
    for k in "ab":
        y = O.normalize_features(g["x_" + k])
        np.testing.assert_array_equal(y.view(np.uint32), g["y_" + k].view(np.uint32))
    c = golden("gcn_cora")
    raw = np.zeros((int(c["n"]), int(c["n_feat"])), np.float32)
    raw[c["feat_row"], c["feat_col"]] = 1.0
    y = O.normalize_features(raw)
    np.testing.assert_array_equal(y[c["feat_row"], c["feat_col"]], c["feat_val"])
    assert np.count_nonzero(y) == c["feat_val"].size


def test_numpy_pairwise_restatement():
    """The oracle's float32 pairwise sum is numpy's add-reduce (what scipy's csr row sum
    runs): bit-exact on random lengths 1..700 and magnitudes."""
    rng = np.random.default_rng(0)
    for _ in range(400):
        n = int(rng.integers(1, 700))
        v = (rng.standard_normal(n) * rng.choice([1e-3, 1.0, 1e3])).astype(np.float32)
        ref = np.add.reduceat(v, np.array([0]))[0]
        mine = np.float32(v[0] + O._np_pairwise_f32(v[1:])) if n > 1 else v[0]
        assert ref.tobytes() == np.float32(mine).tobytes(), n


def test_gcn_spmm_adjacencies_match_reference(golden):
    g = golden("gcn_spmm")
    for name in g["cases"]:
        n = int(g[f"{name}_n"])
        e = g[f"{name}_edges"]
        rowptr, col, val = O.gcn_adjacency(e[:, 0], e[:, 1], n)
        rr, _, rv = _csr_from_ref(g[f"{name}_row"], g[f"{name}_col"], g[f"{name}_val"], n)
        np.testing.assert_array_equal(rowptr, rr)
        assert np.sort(val).tobytes() == np.sort(rv).tobytes()


def test_gcn_cora_logits(golden):
    g = golden("gcn_cora")
    n, nf = int(g["n"]), int(g["n_feat"])
    X = np.zeros((n, nf), np.float32)
    X[g["feat_row"], g["feat_col"].astype(np.int64)] = g["feat_val"]
    rowptr, col, val = _csr_from_ref(g["adj_row"], g["adj_col"], g["adj_val"], n)
    logits = O.gcn_model(rowptr, col, val, X, [g["w0"], g["w1"]], [g["b0"], g["b1"]])
    close(logits, g["logits"])
    assert list(g["state_keys"]) == ["gcn_blocks.gcn0.bias", "gcn_blocks.gcn0.dense.weight",
                                     "gcn_blocks.gcn1.bias", "gcn_blocks.gcn1.dense.weight"]


@pytest.mark.parametrize("impl", ["numpy", "c"])
def test_gcn_spmm_layer_outputs(golden, impl):
    g = golden("gcn_spmm")
    for name, feats in zip(g["cases"], g["feats"]):
        n = int(g[f"{name}_n"])
        rowptr, col, val = _csr_from_ref(g[f"{name}_row"], g[f"{name}_col"], g[f"{name}_val"], n)
        for F in map(int, str(feats).split(",")):
            X = g[f"{name}_F{F}_xq"].astype(np.float32) / 8
            b = g[f"{name}_F{F}_bias"]
            rows = g[f"{name}_F{F}_rows"]
            if impl == "numpy":
                Y = O.spmm_csr(rowptr, col, val, X, b)
            else:
                Y = c_oracle.spmm_csr(rowptr, col, val, X, b)
            close(Y[rows], g[f"{name}_F{F}_y"])


# ------------------------------------------------------------------ GAT
def _dense_adj(row, col, val, n):
    A = np.zeros((n, n), np.float32)
    A[row, col] = val
    return A


@pytest.mark.parametrize("kind", ["dense", "sparse"])
def test_gat_heads_and_model(golden, kind):
    g = golden("gat")
    n = int(g["n"])
    A = _dense_adj(g["adj_row"], g["adj_col"], g["adj_val"], n)
    alpha = float(g["alpha"])
    head = O.gat_sparse_head if kind == "sparse" else O.gat_dense_head
    close(head(g["h"], A, g[f"{kind}_W"][0], g[f"{kind}_a"][0], alpha, True), g[f"{kind}_head0"])
    heads = list(zip(g[f"{kind}_W"], g[f"{kind}_a"]))
    out = O.gat_model(g["h"], A, heads, (g[f"{kind}_outW"], g[f"{kind}_outa"]), alpha,
                      sparse=(kind == "sparse"))
    close(out, g[f"{kind}_logits"])


def test_gat_edge_predicates_and_isolated_rows(golden):
    """Dense layer uses adj > 0, sparse uses adj.nonzero() (layers.py:29 vs :98)."""
    g = golden("gat")
    n = int(g["n"])
    alpha = float(g["alpha"])
    An = _dense_adj(g["neg_row"], g["neg_col"], g["neg_val"], n)
    close(O.gat_dense_head(g["h"], An, g["neg_dense_W"], g["neg_dense_a"], alpha, True),
          g["neg_dense_out"])
    close(O.gat_sparse_head(g["h"], An, g["neg_sparse_W"], g["neg_sparse_a"], alpha, True),
          g["neg_sparse_out"])
    A = _dense_adj(g["adj_row"], g["adj_col"], g["adj_val"], n)
    A[int(g["iso_row"]), :] = 0
    close(O.gat_dense_head(g["h"], A, g["neg_dense_W"], g["neg_dense_a"], alpha, True),
          g["iso_dense_out"])
    sp = O.gat_sparse_head(g["h"], A, g["neg_sparse_W"], g["neg_sparse_a"], alpha, True)
    assert int(g["iso_sparse_raises"]) == 1 and np.isnan(sp[int(g["iso_row"])]).all()


# ------------------------------------------------------------ GraphSAGE
def _sd(g, tag):
    p = f"{tag}_sd_"
    return {k[len(p):]: v for k, v in g.items() if k.startswith(p)}


@pytest.mark.parametrize("tag,agg,gcn", [("mean", "MEAN", False), ("max", "MAX", False),
                                         ("gcn", "MEAN", True)])
def test_sage_forward(golden, tag, agg, gcn):
    g = golden("sage")
    sd = _sd(g, tag)
    agg0 = O.aggregator(g[f"{tag}_neigh_feats"], agg)
    if agg == "MAX":
        np.testing.assert_array_equal(agg0, g[f"{tag}_agg0"])  # int64 indices bit-exact
    else:
        close(agg0, g[f"{tag}_agg0"])
    weights = [sd["sage_blocks.sage_layer0.weight.weight"], sd["sage_blocks.sage_layer1.weight.weight"]]
    emb, logits = O.graphsage_forward(g[f"{tag}_center_feats"], g[f"{tag}_nodes_map"],
                                      g[f"{tag}_neigh_feats"], g[f"{tag}_neigh_map"], weights,
                                      agg, gcn, (sd["dense.weight"], sd["dense.bias"]))
    close(emb, g[f"{tag}_emb"])
    close(logits, g[f"{tag}_logits"])


def test_sage_argmax_rules():
    x = np.array([[[1.0, 2.0], [3.0, 2.0], [3.0, np.nan]]], np.float32)  # [1,3,2]
    np.testing.assert_array_equal(O.aggregator(x, "MAX"), [[1, 2]])


@pytest.mark.parametrize("kind", ["dense", "sparse"])
def test_gat_csr_form_matches_reference_heads(golden, kind):
    """The edge-list restatement (the GPU checker at scale) equals the reference heads."""
    g = golden("gat")
    n = int(g["n"])
    alpha = float(g["alpha"])
    A = _dense_adj(g["adj_row"], g["adj_col"], g["adj_val"], n)
    mask = A > 0 if kind == "dense" else A != 0
    r, c = np.nonzero(mask)
    rowptr, col, _ = O.coo_to_csr(r, c, np.ones(r.size), n)
    W = g[f"{kind}_W"]                      # [H, in, fh]
    a = g[f"{kind}_a"]                      # [H, 2fh]
    H, _, fh = W.shape
    Wall = np.concatenate(list(W), axis=1)  # [in, H*fh]
    wh = g["h"].astype(np.float64) @ Wall
    el, er = O.gat_logits(wh, H, fh, a[:, :fh].reshape(-1), a[:, fh:].reshape(-1))
    out = O.gat_csr(rowptr, col, wh, el, er, H, fh, alpha, kind == "sparse")
    out = np.where(out > 0, out, np.expm1(np.minimum(out, 0)))
    close(out, g[f"{kind}_concat"])


def _han_params(d, layer, M, heads):
    p = f"sd_layers.{layer}."
    gat = [[(d[f"{p}gat_layers.meta_path_model{m}.attentions.AttentionHead{i}.W"],
             d[f"{p}gat_layers.meta_path_model{m}.attentions.AttentionHead{i}.a"])
            for i in range(heads)] for m in range(M)]
    sem = (d[f"{p}semantic_attention.project.0.weight"], d[f"{p}semantic_attention.project.0.bias"],
           d[f"{p}semantic_attention.project.2.weight"])
    return gat, sem


def _han_graphs(d, N, M):
    gs = []
    for m in range(M):
        A = np.zeros((N, N), np.float32)
        A[d[f"g{m}_row"], d[f"g{m}_col"]] = 1
        gs.append(A)
    return gs


def test_han_oracle_matches_reference(golden):
    """HANModel (HAN/models/HAN.py:26-41) restated layer by layer == the reference's logits."""
    d = golden("han")
    N, M, Fin, hid, C = d["dims"]
    heads = d["heads"]
    gs = _han_graphs(d, N, M)
    h = d["h"]
    for layer in range(len(heads)):
        gat, sem = _han_params(d, layer, M, heads[layer])
        h = O.han_layer(gs, h, gat, sem)
        if layer == 0:
            np.testing.assert_allclose(h, d["layer0"], rtol=1e-4, atol=1e-5)
    logits = h @ d["sd_predict.weight"].T.astype(np.float64) + d["sd_predict.bias"]
    np.testing.assert_allclose(logits, d["logits"], rtol=1e-4, atol=1e-5)


def test_graphsage_tree_oracle_matches_reference(golden):
    """GraphSAGE_Pytorch GraphSage / SageGCN / NeighborAggregator restated == reference outputs."""
    d = golden("sagepy")
    Fin, B, h0, h1, k0, k1 = d["dims"]
    layers = [(d[f"sd_gcn.{i}.weight"], d[f"sd_gcn.{i}.aggregator.weight"]) for i in range(2)]
    y = O.graphsage_tree([d["X0"], d["X1"], d["X2"]], layers, [k0, k1])
    np.testing.assert_allclose(y, d["y"], rtol=1e-4, atol=1e-5)
    nb = d["X1"].reshape(B, k0, Fin)
    y2 = O.sage_gcn(d["X0"], nb, d["sumcat_sd_weight"], d["sumcat_sd_aggregator.weight"],
                    neigh="sum", hidden="concat")
    np.testing.assert_allclose(y2, d["sumcat_y"], rtol=1e-4, atol=1e-5)
    y3 = O.neighbor_aggregator(nb, d["biasmean_sd_weight"], d["biasmean_sd_bias"], "mean")
    np.testing.assert_allclose(y3, d["biasmean_y"], rtol=1e-4, atol=1e-5)
    assert int(d["max_raises"]) == 1


# ------------------------------------------------------- GAT block gradients
def _gatgrad_inputs(g, kind):
    n, H, fh = int(g["n"]), int(g["heads"]), int(g["fh"])
    row, col = g["adj_row"].astype(np.int64), g["adj_col"].astype(np.int32)
    order = np.lexsort((col, row))
    row, col = row[order], col[order]
    rowptr = np.concatenate([[0], np.cumsum(np.bincount(row, minlength=n))]).astype(np.int64)
    W = np.concatenate(list(g[f"{kind}_W"]), axis=1)                      # [in, H fh]
    a = g[f"{kind}_a"]                                                    # [H, 2 fh]
    return n, H, fh, rowptr, col, W, a[:, :fh].reshape(-1), a[:, fh:].reshape(-1)


@pytest.mark.parametrize("kind", ["dense", "sparse"])
def test_gat_block_grad_oracle_matches_reference_autograd(golden, kind):
    """oracle_gat_block_grad (the float64 checker of the full-size GAT training test) against
    the reference's own autograd of the 8-head block (layers.py:22-37 dense, :94-131 with
    SpecialSpmmFunction.backward :54-64 sparse; GAT.py:16 concatenation): the block output,
    every head's dW and da, and dh, for the loss sum(block * gy)."""
    g = golden("gatgrad")
    n, H, fh, rowptr, col, W, a_s, a_d = _gatgrad_inputs(g, kind)
    r = c_oracle.gat_block_grad(rowptr, col, g["h"], W, a_s, a_d, g["gy"], H, fh,
                                float(g["alpha"]), kind == "sparse")
    close(r["out"], g[f"{kind}_out"])
    close(r["dW"], np.concatenate(list(g[f"{kind}_dW"]), axis=1))
    da = np.concatenate([r["da_src"].reshape(H, fh), r["da_dst"].reshape(H, fh)], axis=1)
    close(da, g[f"{kind}_da"])
    close(r["dx"], g[f"{kind}_dh"])


def _hash3(seed: int, edge: np.ndarray, head: int) -> np.ndarray:
    """csrc/gat.hip hash3 in numpy uint32 arithmetic (the dropout stream)."""
    M = np.uint64(0xFFFFFFFF)
    e = edge.astype(np.uint64)
    h = np.uint64(seed & 0xFFFFFFFF) ^ ((np.uint64(seed >> 32) * np.uint64(0x27d4eb2f)) & M)
    h = h ^ ((e & M) * np.uint64(0x9e3779b9) & M)
    h = h ^ (((e >> np.uint64(32)) * np.uint64(0x85ebca6b)) & M)
    h = h ^ ((np.uint64(head) * np.uint64(0xc2b2ae35)) & M)
    h = h ^ (h >> np.uint64(16))
    h = (h * np.uint64(0x85ebca6b)) & M
    h = h ^ (h >> np.uint64(13))
    h = (h * np.uint64(0xc2b2ae35)) & M
    h = h ^ (h >> np.uint64(16))
    return h


@pytest.mark.parametrize("sparse", [False, True])
def test_gat_block_grad_oracle_dropout(golden, sparse):
    """With dropout the oracle re-derives the HIP kernels' (seed, CSR edge, head) masks: checked
    against torch float64 autograd of the same block with the mask applied where the reference
    applies F.dropout (after the softmax, layers.py:30 / after the rowsum, :115; inverted,
    scale 1 / (1 - p))."""
    import torch
    g = golden("gatgrad")
    kind = "sparse" if sparse else "dense"
    n, H, fh, rowptr, col, W, a_s, a_d = _gatgrad_inputs(g, kind)
    p, seed, slope = 0.35, 0x1234_5678_9abc, float(g["alpha"])
    r = c_oracle.gat_block_grad(rowptr, col, g["h"], W, a_s, a_d, g["gy"], H, fh, slope, sparse,
                                drop_p=p, drop_seed=seed)
    row = np.repeat(np.arange(n), np.diff(rowptr))
    eid = np.arange(col.size)
    x = torch.tensor(g["h"], dtype=torch.float64, requires_grad=True)
    Wt = torch.tensor(W, dtype=torch.float64, requires_grad=True)
    ast = torch.tensor(a_s, dtype=torch.float64, requires_grad=True)
    adt = torch.tensor(a_d, dtype=torch.float64, requires_grad=True)
    wh = (x @ Wt).view(n, H, fh)
    el = (wh * ast.view(H, fh)).sum(-1)
    er = (wh * adt.view(H, fh)).sum(-1)
    outs = []
    for h in range(H):
        t = el[row, h] + er[col, h]
        z = torch.nn.functional.leaky_relu(t, slope)
        z = -z if sparse else z
        dense = torch.full((n, n), float("-inf"), dtype=torch.float64)
        dense = dense.index_put((torch.from_numpy(row), torch.from_numpy(col.astype(np.int64))), z)
        att = torch.softmax(dense, dim=1)
        keep = (_hash3(seed, eid, h) >> np.uint64(8)).astype(np.float64) / 16777216.0 >= p
        m = torch.zeros((n, n), dtype=torch.float64)
        m[torch.from_numpy(row), torch.from_numpy(col.astype(np.int64))] = \
            torch.from_numpy(keep.astype(np.float64) / (1 - p))
        outs.append(torch.nn.functional.elu((att * m) @ wh[:, h, :]))
    out = torch.cat(outs, dim=1)
    (out * torch.tensor(g["gy"], dtype=torch.float64)).sum().backward()
    close(r["out"], out.detach().numpy(), rtol=1e-9, atol_frac=1e-9)
    close(r["dW"], Wt.grad.numpy(), rtol=1e-9, atol_frac=1e-9)
    close(r["da_src"], ast.grad.numpy(), rtol=1e-9, atol_frac=1e-9)
    close(r["da_dst"], adt.grad.numpy(), rtol=1e-9, atol_frac=1e-9)
    close(r["dx"], x.grad.numpy(), rtol=1e-9, atol_frac=1e-9)
