"""Device-side GCN adjacency preprocessing vs the reference-generated adjacency.

graphneuralnetwork_amd.preprocess restates GCN/data_utils.py:32-35,54-70,78; the
structure must match bit-exactly and the fp32 values too.  Runs on CPU tensors
here (the same torch code runs on the device in bench.py)."""
import numpy as np
import torch

from oracle import gnn_oracle as O


def _check(rowptr_g, col_g, val_g, row, col, val, n):
    rr, rc, rv = O.coo_to_csr(row.astype(np.int64), col, val, n)
    np.testing.assert_array_equal(rowptr_g, rr)
    ko = np.lexsort((col_g, np.repeat(np.arange(n), np.diff(rowptr_g))))
    kr = np.lexsort((rc, np.repeat(np.arange(n), np.diff(rr))))
    np.testing.assert_array_equal(col_g[ko], rc[kr])
    np.testing.assert_array_equal(val_g[ko], rv[kr])


def test_preprocess_matches_reference_fixtures(golden):
    from graphneuralnetwork_amd.preprocess import gcn_normalized_csr
    g = golden("gcn_cora")
    n = int(g["n"])
    csr = gcn_normalized_csr(g["edges"][:, 0], g["edges"][:, 1], n)
    _check(csr.rowptr.numpy(), csr.col.numpy(), csr.val.numpy(), g["adj_row"], g["adj_col"],
           g["adj_val"], n)
    s = golden("gcn_spmm")
    for name in s["cases"]:
        n = int(s[f"{name}_n"])
        e = s[f"{name}_edges"]
        csr = gcn_normalized_csr(e[:, 0], e[:, 1], n)
        _check(csr.rowptr.numpy(), csr.col.numpy(), csr.val.numpy(), s[f"{name}_row"],
               s[f"{name}_col"], s[f"{name}_val"], n)


def test_preprocess_matches_oracle_rmat():
    from graphneuralnetwork_amd.preprocess import gcn_normalized_csr
    from graphneuralnetwork_amd.rmat import rmat_edges
    n = 50_000
    s, d = rmat_edges(n, 400_000, 7)
    csr = gcn_normalized_csr(s, d, n)
    rowptr, col, val = O.gcn_adjacency(s, d, n)
    np.testing.assert_array_equal(csr.rowptr.numpy(), rowptr)
    np.testing.assert_array_equal(csr.col.numpy(), col)  # both ascending within a row
    np.testing.assert_array_equal(csr.val.numpy(), val)


def test_rmat_recipe_nnz():
    """The survey's recipe reproduces its nnz at a small scale deterministically."""
    from graphneuralnetwork_amd.rmat import rmat_edges
    a = rmat_edges(4096, 30000, 0)
    b = rmat_edges(4096, 30000, 0)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert a[0].max() < 4096 and a[1].max() < 4096
