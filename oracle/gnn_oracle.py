"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

A plain-numpy restatement of the reference (kaddly/GraphNeuralNetwork) algorithm
for the GCN / GAT / GraphSAGE aggregation path, used as the *checker* of the
HIP kernels.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it; the product package
(``graphneuralnetwork_amd``) never does and has no CPU fallback.

Parity pinning: the restatement is checked against golden vectors produced by
running the reference's own Python code in this container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``;
``tests/test_oracle_golden.py``).  All arithmetic is float64 (the reference is
fp32 except for the adjacency normalisation, which the reference itself does
in float64 before casting to fp32 at GCN/data_utils.py:65).

Every function cites the reference lines it restates.
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------- graph prep


def _np_pairwise_f32(a: np.ndarray) -> np.float32:
    """numpy's float32 pairwise summation (the add-reduce inner loop, numpy 2.2
    ``FLOAT_pairwise_sum``): fewer than 8 values left to right from -0.0; up to 128 values
    in 8 strided accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the tail
    left to right; longer runs split at n/2 rounded down to a multiple of 8."""
    f = np.float32
    n = a.size
    if n < 8:
        res = f(-0.0)
        for v in a:
            res = f(res + v)
        return res
    if n <= 128:
        r = [f(v) for v in a[:8]]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] = f(r[j] + a[i + j])
            i += 8
        res = f(f(f(r[0] + r[1]) + f(r[2] + r[3])) + f(f(r[4] + r[5]) + f(r[6] + r[7])))
        for v in a[i:]:
            res = f(res + v)
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return f(_np_pairwise_f32(a[:n2]) + _np_pairwise_f32(a[n2:]))


def normalize_features(x: np.ndarray) -> np.ndarray:
    """GCN/data_utils.py:39-51 applied to sp.csr_matrix(x, dtype=float32), then
    torch.Tensor(.toarray()) as load_cora does (:83): the row sum is scipy's
    ``np.add.reduceat`` over the row's stored (nonzero) values in column order -- the first
    value plus numpy's float32 pairwise sum of the rest (``_np_pairwise_f32``); r_inv =
    rowsum ** -1 in float64 with inf -> 0; each value r_inv * x in float64, cast to fp32.
    A zero r_inv zeroes the row to +0.0: scipy's sparse product drops the exact-zero
    products (0 x negative = -0.0 included), so toarray() reads +0.0 there."""
    x = np.asarray(x, dtype=np.float32)
    out = np.zeros_like(x)
    for i in range(x.shape[0]):
        nz = np.flatnonzero(x[i])
        if nz.size == 0:
            continue
        v = x[i, nz]
        s = np.float32(v[0] + _np_pairwise_f32(v[1:])) if v.size > 1 else v[0]
        with np.errstate(divide="ignore"):
            r = np.power(np.float64(s), -1.0)
        if np.isinf(r):
            continue          # r_inv = 0: every product is an exact zero, dropped -> +0.0
        out[i, nz] = (r * v.astype(np.float64)).astype(np.float32)
    return out


def coalesce_counts(src: np.ndarray, dst: np.ndarray, n: int):
    """COO edge list -> unique (row, col, count) sorted row-major.

    Restates ``sp.coo_matrix((np.ones(E), (e0, e1)))`` followed by the implicit
    duplicate summation of its first CSR conversion (GCN/data_utils.py:32-35).
    """
    key = src.astype(np.int64) * n + dst.astype(np.int64)
    uk, cnt = np.unique(key, return_counts=True)
    return (uk // n).astype(np.int64), (uk % n).astype(np.int64), cnt.astype(np.float64)


def symmetrize_max(row, col, w, n: int):
    """A_sym = A + A^T.multiply(A^T > A) - A.multiply(A^T > A)  (GCN/data_utils.py:35).

    For non-negative A this is the element-wise maximum of A and A^T.
    Returns unique (row, col, value) sorted row-major.
    """
    r = np.concatenate([row, col])
    c = np.concatenate([col, row])
    v = np.concatenate([w, w])
    key = r * n + c
    order = np.lexsort((-v, key))  # per key, largest value first
    key, v = key[order], v[order]
    first = np.ones(key.size, dtype=bool)
    first[1:] = key[1:] != key[:-1]
    key, v = key[first], v[first]
    return key // n, key % n, v


def add_self_loops(row, col, val, n: int):
    """adj + sp.eye(N)  (GCN/data_utils.py:78): adds 1.0 on the diagonal (float64)."""
    key = np.concatenate([row * n + col, np.arange(n, dtype=np.int64) * (n + 1)])
    v = np.concatenate([val.astype(np.float64), np.ones(n)])
    uk, inv = np.unique(key, return_inverse=True)
    out = np.zeros(uk.size)
    np.add.at(out, inv, v)
    return uk // n, uk % n, out


def normalize_adj(row, col, val, n: int):
    """A_hat = (A D^-1/2)^T D^-1/2 = D^-1/2 A^T D^-1/2  (GCN/data_utils.py:54-60).

    D = rowsum(A) in float64, d^-1/2 with inf -> 0.  Entry (i, j) of the result
    is (A[j, i] * d[i]) * d[j]; returned as (row, col, float64 value) sorted
    row-major (row = output node i).
    """
    rowsum = np.zeros(n)
    np.add.at(rowsum, row, val)
    with np.errstate(divide="ignore"):
        d = np.power(rowsum, -0.5)
    d[np.isinf(d)] = 0.0
    # transpose: entry (i=col, j=row) = (val * d[col]) * d[row]
    r_t, c_t = col, row
    v_t = (val * d[col]) * d[row]
    order = np.lexsort((c_t, r_t))
    return r_t[order], c_t[order], v_t[order]


def gcn_adjacency(src: np.ndarray, dst: np.ndarray, n: int):
    """Full reference pipeline C3 -> +I -> C2 -> fp32 (GCN/data_utils.py:27-36,54-70,78,85).

    Returns CSR (rowptr int64, col int32, val float32).
    """
    r, c, w = coalesce_counts(src, dst, n)
    r, c, w = symmetrize_max(r, c, w, n)
    r, c, w = add_self_loops(r, c, w, n)
    r, c, w = normalize_adj(r, c, w, n)
    return coo_to_csr(r, c, w.astype(np.float32), n)


def coo_to_csr(row, col, val, n_rows: int):
    """Stable row sort of COO triplets (duplicates kept)."""
    row = np.asarray(row, dtype=np.int64)
    order = np.argsort(row, kind="stable")
    rowptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(np.bincount(row, minlength=n_rows), out=rowptr[1:])
    return rowptr, np.asarray(col)[order].astype(np.int32), np.asarray(val)[order]


# ---------------------------------------------------------------------- GCN


def spmm_csr(rowptr, col, val, x, bias=None):
    """Y = A X (+ bias), float64 accumulation  (torch.spmm at GCN/GCN.py:43, + bias :45)."""
    x = np.asarray(x, dtype=np.float64)
    n_rows = rowptr.size - 1
    contrib = np.asarray(val, dtype=np.float64)[:, None] * x[np.asarray(col, dtype=np.int64)]
    y = np.zeros((n_rows, x.shape[1]))
    deg = np.diff(rowptr)
    nz = deg > 0
    if contrib.shape[0]:
        y[nz] = np.add.reduceat(contrib, rowptr[:-1][nz], axis=0)
    if bias is not None:
        y = y + np.asarray(bias, dtype=np.float64)
    return y


def gcn_layer(rowptr, col, val, x, weight, bias):
    """Graph_conv_layer.forward (GCN/GCN.py:41-47): spmm(A, X W^T) + b."""
    support = np.asarray(x, np.float64) @ np.asarray(weight, np.float64).T
    return spmm_csr(rowptr, col, val, support, bias)


def gcn_model(rowptr, col, val, x, weights, biases):
    """GCN_Model.forward in eval mode (GCN/GCN.py:21-27): gcn -> relu (-> dropout=id) -> ... -> gcn."""
    h = np.asarray(x, np.float64)
    for i, (w, b) in enumerate(zip(weights, biases)):
        h = gcn_layer(rowptr, col, val, h, w, b)
        if i != len(weights) - 1:
            h = np.maximum(h, 0.0)
    return h


# ---------------------------------------------------------------------- GAT


def _leaky(x, alpha):
    return np.where(x > 0, x, alpha * x)


def _elu(x):
    return np.where(x > 0, x, np.expm1(np.minimum(x, 0)))


def gat_dense_head(h, adj_dense, W, a, alpha, concat):
    """GraphAttentionLayer.forward, eval mode (GAT/models/layers.py:22-37).

    e_ij = LeakyReLU(a[:F].Wh_i + a[F:].Wh_j); masked where adj <= 0 with -9e15;
    row softmax; h' = att . Wh; ELU if concat.  A row with no edge degenerates
    to a uniform average over all N rows (every logit is -9e15).
    """
    Wh = np.asarray(h, np.float64) @ np.asarray(W, np.float64)
    F = Wh.shape[1]
    a = np.asarray(a, np.float64).reshape(-1)
    el = Wh @ a[:F]
    er = Wh @ a[F:]
    e = _leaky(el[:, None] + er[None, :], alpha)
    e = np.where(np.asarray(adj_dense) > 0, e, -9e15)
    e = e - e.max(axis=1, keepdims=True)
    p = np.exp(e)
    att = p / p.sum(axis=1, keepdims=True)
    out = att @ Wh
    return _elu(out) if concat else out


def gat_sparse_head(h, adj_dense, W, a, alpha, concat):
    """SpGraphAttentionLayer.forward, eval mode (GAT/models/layers.py:94-131).

    edges = adj.nonzero(); edge_e = exp(-LeakyReLU(a.[Wh_i || Wh_j])) (no max
    subtraction, as the reference); h' = (sum_j edge_e Wh_j) / (sum_j edge_e);
    a row without edges gives 0/0 = NaN (the reference then fails its
    ``assert not isnan``); ELU if concat.
    """
    Wh = np.asarray(h, np.float64) @ np.asarray(W, np.float64)
    F = Wh.shape[1]
    a = np.asarray(a, np.float64).reshape(-1)
    ii, jj = np.nonzero(np.asarray(adj_dense))
    s = Wh[ii] @ a[:F] + Wh[jj] @ a[F:]
    ee = np.exp(-_leaky(s, alpha))
    n = Wh.shape[0]
    rowsum = np.zeros(n)
    np.add.at(rowsum, ii, ee)
    acc = np.zeros_like(Wh)
    np.add.at(acc, ii, ee[:, None] * Wh[jj])
    with np.errstate(invalid="ignore", divide="ignore"):
        out = acc / rowsum[:, None]
    return _elu(out) if concat else out


def gat_model(h, adj_dense, heads, out_head, alpha, sparse: bool):
    """GATBase.forward, eval mode (GAT/models/GAT.py:14-18): concat heads -> out_att -> ELU."""
    f = gat_sparse_head if sparse else gat_dense_head
    x = np.concatenate([f(h, adj_dense, W, a, alpha, True) for W, a in heads], axis=1)
    W, a = out_head
    return _elu(f(x, adj_dense, W, a, alpha, False))


# ---------------------------------------------------------------- GraphSAGE


def aggregator(neigh_feat, agg_func="MEAN"):
    """Aggregator (GraphSAGE/graph_utils.py:4-11).

    MEAN -> mean over dim 1 (float64 here); MAX -> argmax over dim 1 as int64:
    first maximal position, a NaN counts as the maximum (torch.argmax rule).
    """
    x = np.asarray(neigh_feat)
    if agg_func == "MEAN":
        return x.astype(np.float64).mean(axis=1)
    if agg_func == "MAX":
        nan = np.isnan(x)
        arg = np.argmax(np.where(nan, -np.inf, x), axis=1)
        has_nan = nan.any(axis=1)
        first_nan = np.argmax(nan, axis=1)
        return np.where(has_nan, first_nan, arg).astype(np.int64)
    if agg_func == "MAXPOOL":
        # value max-pool, BASELINE north_star "mean/max-pool": the .values of
        # neighbor_feature.max(dim=1) (GraphSAGE_Pytorch/models/Aggregator.py:23-24); a NaN
        # anywhere in the slice propagates (torch.max rule)
        return x.astype(np.float64).max(axis=1)
    raise RuntimeError("unknown agg_func")


def sage_layer(self_feats, agg_feats, weight, gcn=False):
    """SageLayer.forward (GraphSAGE/GraphSAGE.py:15-20): relu(W . cat[self, agg])."""
    agg = np.asarray(agg_feats, np.float64)
    comb = agg if gcn else np.concatenate([np.asarray(self_feats, np.float64), agg], axis=1)
    return np.maximum(comb @ np.asarray(weight, np.float64).T, 0.0)


def graphsage_forward(center_feats, center_nodes_map, neigh_feats, neigh_nodes_map, weights,
                      agg_func="MEAN", gcn=False, dense=None):
    """GraphSAGE.forward, supervised branch (GraphSAGE/GraphSAGE.py:42-53)."""
    num_layers = len(weights)
    cf = np.asarray(center_feats, np.float64)
    nf = np.asarray(neigh_feats, np.float64)
    feats = None
    for i, w in enumerate(weights):
        agg = aggregator(nf, agg_func)
        feats = sage_layer(cf, agg, w, gcn)
        if i != num_layers - 1:
            cm = np.asarray(center_nodes_map[i])
            nm = np.asarray(neigh_nodes_map[i])
            cf = feats[cm[cm != -1]]
            nf = feats[nm[nm[:, 0] != -1, :]]
    classes = None
    if dense is not None:
        Wd, bd = dense
        classes = feats @ np.asarray(Wd, np.float64).T + np.asarray(bd, np.float64)
    return feats, classes


def sage_gather_aggregate(table, idx, agg_func="MEAN"):
    """Fused gather + Aggregator: Aggregator(embedding(table, idx)) (GraphSAGE/GraphSAGE.py:47-49 + graph_utils.py:6,8)."""
    return aggregator(np.asarray(table)[np.asarray(idx)], agg_func)


def sage_layer_adj_nodes(nodes, adj_lists, num_layers, num_neighs, is_gcn, rng):
    """get_layer_adj_nodes (GraphSAGE/data_utils.py:82-124), restated with Python sets and a
    ``random.Random``-compatible ``rng`` (the draws and set orders ARE CPython's own, so this
    is exact for small cases; quadratic like the reference's per-node union).

    Per layer i, per node of the layer (a list for i = 0, the previous layer's set after):
    sample ``k`` of ``list(adj_lists[node])`` (rng.sample if deg > k else rng.choices, :91-94),
    append the node in gcn mode else add it to the layer set (:95-98), then
    ``layer = layer.union(set(sample))`` (:100).  Outputs (:104-123), deepest layer first:
    global ids for the last layer, positions in the next layer's enumeration for the others,
    -1 padded to the last layer's length.  Returns (neigh [L][P][k'], center [L][P]) lists.
    """
    layer_neigh, layer_map = [], []
    centers = [list(nodes)]
    cur = nodes
    for i in range(num_layers):
        pos, samples, layer = {}, [], set()
        for idx, node in enumerate(cur):
            pos[node] = idx
            nb = list(adj_lists[node])
            s = rng.sample(nb, k=num_neighs) if len(nb) > num_neighs else \
                rng.choices(nb, k=num_neighs)
            if is_gcn:
                s.append(node)
            else:
                layer.add(node)
            samples.append(s)
            layer = layer.union(set(s))
        layer_neigh.append(samples)
        layer_map.append(pos)
        cur = layer
        centers.append(list(cur))
    neigh_out, center_out = [], []
    pad = len(layer_neigh[-1])
    for i in reversed(range(num_layers)):
        if i == num_layers - 1:
            neigh_out.append([list(r) for r in layer_neigh[i]])
            center_out.append(list(centers[i]))
        else:
            m = layer_map[i + 1]
            rows = [[m[v] for v in r] for r in layer_neigh[i]]
            width = len(rows[0])
            neigh_out.append(rows + [[-1] * width] * (pad - len(rows)))
            cm = [m[v] for v in centers[i]]
            center_out.append(cm + [-1] * (pad - len(cm)))
    return neigh_out, center_out


def gat_csr(rowptr, col, wh, el, er, heads, fh, slope, sparse: bool, empty_fill=None):
    """Edge-list form of both GAT layers for H heads at once, float64.

    dense  (layers.py:25-32): out_i = sum_j softmax_j(LeakyReLU(el_i + er_j)) Wh_j,
           edgeless row -> ``empty_fill`` (the uniform average over all rows);
    sparse (layers.py:105-122): out_i = sum_j exp(-LeakyReLU(.)) Wh_j / sum_j exp(-LeakyReLU(.)).
    Wh [N, H*fh]; el, er [N, H].  No activation.
    """
    wh = np.asarray(wh, np.float64).reshape(-1, heads, fh)
    el = np.asarray(el, np.float64)
    er = np.asarray(er, np.float64)
    n = rowptr.size - 1
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    col = np.asarray(col, np.int64)
    s = _leaky(el[rows] + er[col], slope)                     # [E, H]
    if sparse:
        p = np.exp(-s)
    else:
        mx = np.full((n, heads), -np.inf)
        np.maximum.at(mx, rows, s)
        p = np.exp(s - mx[rows])
    den = np.zeros((n, heads))
    np.add.at(den, rows, p)
    num = np.zeros((n, heads, fh))
    np.add.at(num, rows, p[:, :, None] * wh[col])
    with np.errstate(invalid="ignore", divide="ignore"):
        out = num / den[:, :, None]
    out = out.reshape(n, heads * fh)
    if not sparse:
        empty = np.diff(rowptr) == 0
        if empty.any():
            fill = wh.reshape(n, -1).mean(0) if empty_fill is None else empty_fill
            out[empty] = fill
    return out


def gat_logits(wh, heads, fh, a_src, a_dst):
    """el = a_src . Wh_i, er = a_dst . Wh_j per head (layers.py:25-26, :105-108)."""
    w = np.asarray(wh, np.float64).reshape(-1, heads, fh)
    return (w * np.asarray(a_src, np.float64).reshape(heads, fh)).sum(-1), \
           (w * np.asarray(a_dst, np.float64).reshape(heads, fh)).sum(-1)


# ------------------------------------------------------------------ HAN
def han_gatconv(h, adj_dense, heads, alpha=0.2, out_head=None):
    """GATConv.forward, eval mode (HAN/models/NodeAttention.py:59-62): concat of the
    ELU'd dense heads, then ELU(out_att) -- or, without out_att, ELU once more."""
    x = np.concatenate([gat_dense_head(h, adj_dense, W, a, alpha, True) for W, a in heads], 1)
    if out_head is not None:
        return _elu(gat_dense_head(x, adj_dense, out_head[0], out_head[1], alpha, False))
    return _elu(x)


def han_semantic_attention(z, w1, b1, w2):
    """SemanticAttention.forward (HAN/models/SemanticAttention.py:15-20):
    beta = softmax_M(mean_N(tanh(z W1^T + b1) W2^T)); out = sum_M beta_M z[:, M]."""
    z = np.asarray(z, np.float64)
    w = (np.tanh(z @ np.asarray(w1, np.float64).T + np.asarray(b1, np.float64))
         @ np.asarray(w2, np.float64).T).mean(0)                       # (M, 1)
    beta = np.exp(w - w.max(0)) / np.exp(w - w.max(0)).sum(0)
    return (beta[None] * z).sum(1)


def han_layer(gs, h, gat_heads, sem):
    """HANLayer.forward (HAN/models/HAN.py:17-23): one GATConv per metapath graph,
    stacked (N, M, D*K), semantic attention over M."""
    z = np.stack([han_gatconv(h, g, heads) for g, heads in zip(gs, gat_heads)], 1)
    return han_semantic_attention(z, *sem)


# -------------------------------------------------- GraphSAGE_Pytorch
def neighbor_aggregator(nb, weight, bias=None, method="mean"):
    """NeighborAggregator.forward (GraphSAGE_Pytorch/models/Aggregator.py:18-33):
    mean / sum over dim 1, then @ weight (+ bias)."""
    nb = np.asarray(nb, np.float64)
    a = nb.mean(1) if method == "mean" else nb.sum(1)
    out = a @ np.asarray(weight, np.float64)
    return out if bias is None else out + np.asarray(bias, np.float64)


def sage_gcn(src, nb, weight, agg_weight, agg_bias=None, neigh="mean", hidden="sum", relu=True):
    """SageGCN.forward (GraphSAGE_Pytorch/models/SageGCN.py:24-37)."""
    nh = neighbor_aggregator(nb, agg_weight, agg_bias, neigh)
    sh = np.asarray(src, np.float64) @ np.asarray(weight, np.float64)
    out = sh + nh if hidden == "sum" else np.concatenate([sh, nh], 1)
    return np.maximum(out, 0) if relu else out


def graphsage_tree(feats, layers, nbrs):
    """GraphSage.forward (GraphSAGE_Pytorch/models/GraphSage.py:20-31): layer l folds hop
    features pairwise (hop, hop+1 viewed as [n_hop, k_hop, F]); last layer has no ReLU.
    layers: [(weight, agg_weight)] per layer."""
    hidden = [np.asarray(f, np.float64) for f in feats]
    L = len(nbrs)
    for l in range(L):
        w, aw = layers[l]
        hidden = [sage_gcn(hidden[hop], hidden[hop + 1].reshape(len(hidden[hop]), nbrs[hop], -1),
                           w, aw, relu=l < L - 1) for hop in range(L - l)]
    return hidden[0]
