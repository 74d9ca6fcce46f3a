"""XCD-sliced hub staging plan (graph.xcd_hub_coo): host-side structure and algebra.

The plan regroups each row's sum A_i. X into [edges left in place] + [one partial row per
(row, XCD slice) item]; here the two edge lists are checked on the CPU against the oracle
SpMM (float64), and their layout against what the GPU launch relies on (item positions
dealt to XCDs in workgroups of 4, 2..chunk edges per item, refs after the row's own edges).
"""
import numpy as np
import pytest
import torch

from oracle import gnn_oracle as O

XCDS, W = 8, 4


def _hub_rename(col, n, k):
    """col_hub as hub.hip builds it: the k highest in-degree columns (ties by ascending id)
    renamed -1-rank."""
    deg = np.bincount(col, minlength=n)
    hub = np.lexsort((np.arange(n), -deg))[:k]
    rank = np.full(n, -1, np.int64)
    rank[hub] = np.arange(k)
    ch = np.where(rank[col] >= 0, -1 - rank[col], col)
    return hub, ch


def _graph(n=3000, e=60000, seed=0):
    from graphneuralnetwork_amd.rmat import rmat_edges
    s, d = rmat_edges(n, e, seed)
    return O.gcn_adjacency(s, d, n)


def _decode(cols, X, B):
    return np.where(cols[:, None] >= 0, X[np.maximum(cols, 0)], B[np.maximum(-1 - cols, 0)])


def _csr_spmm(rows, cols, vals, n_rows, src):
    """sum over edges of vals * src-row, per row (float64)."""
    out = np.zeros((n_rows, src.shape[1]))
    np.add.at(out, rows, vals[:, None].astype(np.float64) * src)
    return out


@pytest.mark.parametrize("k,min_deg,chunk,phases,item_k,small_item", [
    (64, 16, 8, 1, None, None), (200, 2, 4, 1, None, None), (500, 64, 128, 1, None, None),
    (3000, 1, 4, 1, None, None), (3000, 1, 5, 1, None, None), (500, 16, 8, 2, None, None),
    (3000, 2, 4, 4, None, None), (3000, 2, 8, 1, 100, None), (500, 16, 8, 2, 64, None),
    (500, 64, 128, 1, None, 3), (3000, 32, 8, 1, None, 4), (500, 10 ** 9, 16, 1, None, 2)])
@pytest.mark.parametrize("group", [1, 4])
def test_xcd_plan_algebra_and_layout(monkeypatch, k, min_deg, chunk, phases, item_k, small_item,
                                     group):
    from graphneuralnetwork_amd import graph as G
    from graphneuralnetwork_amd.graph import xcd_hub_coo
    monkeypatch.setattr(G, "XCD_SLICE_GROUP", group)
    S = XCDS * phases
    gs = group if (item_k or k) >= S * group else 1  # hub rank r in slice (r // gs) % S
    rowptr, col, val = _graph()
    n = rowptr.size - 1
    hub, ch = _hub_rename(col, n, k)
    res = xcd_hub_coo(torch.from_numpy(rowptr), torch.from_numpy(ch.astype(np.int32)),
                      torch.from_numpy(val), k, min_deg, chunk, phases=phases, item_k=item_k,
                      small_item=small_item)
    assert res is not None
    (ir, ic, iv, n_pos, n_items), (rr, rc, rv), pos_row = res
    ir, ic, iv, rr, rc, rv = (t.numpy() for t in (ir, ic, iv, rr, rc, rv))
    # layout: positions fill whole workgroups of every XCD; an item only reads its slice
    # (slice = (rank // gs) % (XCDS * phases), on XCD slice % XCDS), the phases in launch order
    assert n_pos % (XCDS * W) == 0
    assert ((ic < 0) & (ic >= -(item_k or k))).all()
    sl = ((-1 - ic) // gs) % S
    np.testing.assert_array_equal(sl % XCDS, (ir // W) % XCDS)
    o = np.argsort(ir, kind="stable")
    assert (np.diff((sl // XCDS)[o]) >= 0).all()
    cnt = np.bincount(ir, minlength=n_pos)
    assert cnt.min() >= 2 and cnt.max() <= chunk
    pads = (iv == 0) & (np.bincount(ir, weights=(iv != 0), minlength=n_pos)[ir] == 0)
    assert n_pos - n_items == len(np.unique(ir[pads]))
    # refs point at partial rows k .. k + n_pos - 1, one per real item
    refs = rc < -k
    assert refs.sum() == n_items and (rv[refs] == 1.0).all()
    assert (-1 - rc[refs] - k < n_pos).all()
    # every original edge appears exactly once (in an item or left in place), CSR order kept
    deg = np.diff(rowptr)
    rows_e = np.repeat(np.arange(n), deg)
    kept = ~refs
    moved_rows = np.empty(ir.size, np.int64)
    pos_row = pos_row.numpy()
    np.testing.assert_array_equal(pos_row[-1 - rc[refs] - k], rr[refs])
    moved_rows = pos_row[ir[~pads]]
    both = np.concatenate([np.stack([rr[kept], rc[kept]]), np.stack([moved_rows, ic[~pads]])], 1)
    orig = np.stack([rows_e, ch])
    np.testing.assert_array_equal(np.lexsort(both[::-1]).size, orig.shape[1])
    np.testing.assert_array_equal(both[:, np.lexsort(both[::-1])], orig[:, np.lexsort(orig[::-1])])
    # items of rows below min_deg only for (row, slice) groups of >= small_item hub edges
    deg_item = deg[moved_rows]
    grp = moved_rows * S + ((-1 - ic[~pads]) // gs) % S
    _, inv, gsize = np.unique(grp, return_inverse=True, return_counts=True)
    low = deg_item < min_deg
    if small_item is None:
        assert not low.any()
    else:
        assert (gsize[inv][low] >= small_item).all() and low.any()
    # rest rows: own edges in CSR order before the partial refs
    order = np.argsort(rr, kind="stable")
    rs, rcs = rr[order], rc[order]
    for r in np.unique(rs[rcs < -k])[:50]:
        seg = rcs[rs == r]
        is_ref = seg < -k
        assert not (is_ref[:-1] & ~is_ref[1:]).any()
    # algebra: pass 1 over the staged table, pass 2 over [table | partials] and X == A . X
    rng = np.random.default_rng(1)
    X = rng.standard_normal((n, 5))
    T = X[hub]
    P = _csr_spmm(ir, ic, iv, n_pos, _decode(ic, X, T))
    B = np.concatenate([T, P])
    Y = _csr_spmm(rr, rc, rv, n, _decode(rc, X, B))
    np.testing.assert_allclose(Y, O.spmm_csr(rowptr, col, val, X), rtol=1e-12, atol=1e-12)


def test_xcd_plan_none_without_items():
    from graphneuralnetwork_amd.graph import xcd_hub_coo
    rowptr, col, val = _graph(500, 3000, 2)
    n = rowptr.size - 1
    _, ch = _hub_rename(col, n, 16)
    assert xcd_hub_coo(torch.from_numpy(rowptr), torch.from_numpy(ch.astype(np.int32)),
                       torch.from_numpy(val), 16, 10 ** 9, 8) is None
    with pytest.raises(ValueError):
        xcd_hub_coo(torch.from_numpy(rowptr), torch.from_numpy(ch.astype(np.int32)),
                    torch.from_numpy(val), 4, 2, 8)
    with pytest.raises(ValueError):
        xcd_hub_coo(torch.from_numpy(rowptr), torch.from_numpy(ch.astype(np.int32)),
                    torch.from_numpy(val), 16, 2, 3)
    with pytest.raises(ValueError):  # fewer hub rows than slices
        xcd_hub_coo(torch.from_numpy(rowptr), torch.from_numpy(ch.astype(np.int32)),
                    torch.from_numpy(val), 16, 2, 8, phases=4)


@pytest.mark.parametrize("max_deg,cost", [(1, 4), (8, 16), (64, 256), (128, 256)])
def test_task_ranges_invariants(max_deg, cost):
    """graph.task_ranges (CPU torch ops): tasks cover exactly the rows of degree <= max_deg,
    in order, without overlap; each holds <= 63 consecutive rows of one run and at most
    cost + max_deg + 1 (edges + rows)."""
    import numpy as np
    import torch
    from graphneuralnetwork_amd.graph import TASK_ROWS, task_ranges
    rng = np.random.default_rng(max_deg + cost)
    deg = rng.zipf(1.7, 20000).clip(0, 5000) - 1
    deg[rng.random(deg.size) < 0.15] = 0
    deg[5000:5200] = 0
    rowptr = torch.from_numpy(np.concatenate([[0], np.cumsum(deg)]).astype(np.int64))
    t = task_ranges(rowptr, max_deg, cost).numpy().reshape(-1, 2)
    covered = np.zeros(deg.size, bool)
    prev_end = 0
    for b, e in t:
        assert prev_end <= b < e <= deg.size and e - b <= TASK_ROWS
        assert not covered[b:e].any()
        covered[b:e] = True
        assert (deg[b:e] <= max_deg).all()
        assert int((deg[b:e] + 1).sum()) <= cost + max_deg + 1
        prev_end = e
    np.testing.assert_array_equal(covered, deg <= max_deg)
    assert task_ranges(torch.zeros(1, dtype=torch.int64), max_deg, cost).numel() == 0


@pytest.mark.parametrize("rows,prefix", [(True, None), (False, None), (False, 300),
                                         (True, 1000)])
def test_degree_order_bit_identical_and_hub_prefix(rows, prefix):
    """graph.degree_order (CPU torch ops): A' = P A P^T (or A P^T) with each row's edges in
    their CSR order, so A' X' equals the original product bit for bit (permuted); the
    in-degree ranking of hub.hip (descending, ties by ascending id) is then the identity.
    ``prefix``: the first ``prefix`` ids are the full order's, the rest ascending ids."""
    from graphneuralnetwork_amd.graph import CsrGraph, degree_order
    rowptr, col, val = _graph(4000, 50000, 3)
    n = rowptr.size - 1
    g = CsrGraph(torch.from_numpy(rowptr), torch.from_numpy(col.astype(np.int32)),
                 torch.from_numpy(val), n, n)
    o = degree_order(g, rows=rows, prefix=prefix)
    perm, inv = o.perm.numpy(), o.inv.numpy()
    if prefix is not None:
        full = degree_order(g, rows=False).perm.numpy()
        np.testing.assert_array_equal(perm[:prefix], full[:prefix])
        np.testing.assert_array_equal(perm[prefix:], np.sort(full[prefix:]))
    np.testing.assert_array_equal(inv[perm], np.arange(n))
    gp = o.graph
    X = np.random.default_rng(5).standard_normal((n, 6))
    Y = O.spmm_csr(rowptr, col, val, X)
    Yp = O.spmm_csr(gp.rowptr.numpy(), gp.col.numpy(), gp.val.numpy(), X[perm])
    np.testing.assert_array_equal(Yp, Y[perm] if rows else Y)
    hub, _ = _hub_rename(gp.col.numpy(), n, 300)
    np.testing.assert_array_equal(hub, np.arange(300))
    if rows:
        np.testing.assert_array_equal(o.unpermute_rows(torch.from_numpy(Yp)).numpy(), Y)


def test_xcd_direct_plan_algebra():
    """XcdHubPlan.direct on a degree-ordered graph: pass 1 gathers the items' hub rows
    straight from X (hub rank = X row), pass 2 reads X and a separate partial-row buffer
    (-1-pos); together they equal A' X' (float64)."""
    from graphneuralnetwork_amd.graph import (CsrGraph, HubPlan, XcdHubPlan, degree_order,
                                              from_coo, xcd_hub_coo)
    rowptr, col, val = _graph(3000, 60000, 0)
    n = rowptr.size - 1
    g = CsrGraph(torch.from_numpy(rowptr), torch.from_numpy(col.astype(np.int32)),
                 torch.from_numpy(val), n, n)
    gp = degree_order(g).graph
    k = 500
    c = gp.col.to(torch.int64)
    col_hub = torch.where(c < k, -1 - c, c).to(torch.int32)
    (ir, ic, iv, n_pos, n_items), (rr, rc, rv), pos_row = xcd_hub_coo(
        gp.rowptr, col_hub, gp.val, k, 16, 8)
    hp = HubPlan(torch.arange(k), col_hub, torch.zeros(1, dtype=torch.int32))
    xp = XcdHubPlan(hp, from_coo(ir, ic, iv, n_pos, k, check=False),
                    from_coo(rr, rc, rv, n, n, check=False),
                    n_items, 16, 8, pos_row)
    assert xp.prefix
    items, rest = xp.direct()
    assert int(items.col.min()) >= 0 and int(items.col.max()) < k
    assert int(rest.col.min()) >= -n_pos
    X = np.random.default_rng(6).standard_normal((n, 4))
    ipr = items.rowptr.numpy()
    P = _csr_spmm(np.repeat(np.arange(n_pos), np.diff(ipr)), items.col.numpy(),
                  items.val.numpy(), n_pos, X[items.col.numpy()])
    rpr, rcol = rest.rowptr.numpy(), rest.col.numpy()
    src = np.where(rcol[:, None] >= 0, X[np.maximum(rcol, 0)], P[np.maximum(-1 - rcol, 0)])
    Y = _csr_spmm(np.repeat(np.arange(n), np.diff(rpr)), rcol, rest.val.numpy(), n, src)
    want = O.spmm_csr(gp.rowptr.numpy(), gp.col.numpy(), gp.val.numpy(), X)
    np.testing.assert_allclose(Y, want, rtol=1e-12, atol=1e-12)


def test_sampler_degree_ordered_dataset():
    """sampler.degree_ordered (CPU torch ops): node v of the relabelled dataset is node
    perm[v]; every row keeps its neighbour set (renamed) in ascending order; the table rows
    follow; degrees are non-increasing."""
    from graphneuralnetwork_amd.rmat import rmat_edges
    from graphneuralnetwork_amd.sampler import degree_ordered, symmetric_adjacency
    n = 3000
    s, d = rmat_edges(n, 30000, 4)
    adj = symmetric_adjacency(s, d, n)
    table = torch.randn(n, 5)
    g2, t2, o = degree_ordered(adj, table)
    perm, inv = o.perm.numpy(), o.inv.numpy()
    rp, c = adj.rowptr.numpy(), adj.col.numpy()
    rp2, c2 = g2.rowptr.numpy(), g2.col.numpy()
    assert (np.diff(np.diff(rp2)) <= 0).all()
    for v in range(n):
        got = c2[rp2[v]:rp2[v + 1]]
        want = np.sort(inv[c[rp[perm[v]]:rp[perm[v] + 1]]])
        np.testing.assert_array_equal(got, want)
    assert torch.equal(t2, table[o.perm])
