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
