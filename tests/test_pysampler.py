"""CPython-exact GraphSAGE sampler (csrc/pysample.cpp, graphneuralnetwork_amd/pysampler.py).

Pinned by tests/golden/pysampler.npz (the reference's get_layer_adj_nodes run under a
seeded global ``random``, tests/golden/make_golden.py part_pysampler): index maps
bit-exact and the generator left in the same state.  The oracle restatement
(oracle.gnn_oracle.sage_layer_adj_nodes) is pinned by the same vectors and then checks
the native sampler on more shapes.  Host-only code: no GPU needed (except collate_fn).
"""
import ctypes
import random
from collections import defaultdict
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import gnn_oracle as O

GOLD = Path(__file__).resolve().parent / "golden" / "pysampler.npz"
GRAPHS = ("small", "mid")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def _adj_lists(g, name):
    """The reference's defaultdict(set) rebuilt from the stored pair stream (data_utils.py:36-37)."""
    adj = defaultdict(set)
    for a, b in g[f"{name}_pairs"].tolist():
        adj[a].add(b)
        adj[b].add(a)
    return adj


def _rng_at(words):
    r = random.Random()
    r.setstate((3, tuple(int(w) for w in words), None))
    return r


def _cases(g):
    c = 0
    while f"case{c}_meta" in g:
        gi, L, K, gcn, seed = (int(v) for v in g[f"case{c}_meta"])
        yield c, GRAPHS[gi], L, K, bool(gcn)
        c += 1


def test_adjacency_order_from_pairs(gold):
    from graphneuralnetwork_amd.pysampler import PyAdjacency
    for name in GRAPHS:
        n = int(gold[f"{name}_n"])
        pa = PyAdjacency.from_pairs(gold[f"{name}_pairs"][:, 0], gold[f"{name}_pairs"][:, 1], n)
        np.testing.assert_array_equal(pa.rowptr, gold[f"{name}_adj_ptr"])
        np.testing.assert_array_equal(pa.nbr, gold[f"{name}_adj_nbr"])
        # and reading the reference's own sets gives the same lists
        pb = PyAdjacency.from_adj_lists(_adj_lists(gold, name), n)
        np.testing.assert_array_equal(pb.nbr, pa.nbr)


def test_oracle_restatement_matches_reference(gold):
    adjs = {n: _adj_lists(gold, n) for n in GRAPHS}
    for c, name, L, K, gcn in _cases(gold):
        r = _rng_at(gold[f"case{c}_state0"])
        neigh, center = O.sage_layer_adj_nodes(gold[f"case{c}_nodes"].tolist(), adjs[name], L, K,
                                               gcn, r)
        np.testing.assert_array_equal(np.asarray(neigh), gold[f"case{c}_neigh"])
        np.testing.assert_array_equal(np.asarray(center), gold[f"case{c}_center"])
        np.testing.assert_array_equal(np.asarray(r.getstate()[1], np.uint32),
                                      gold[f"case{c}_state1"])


def test_native_sampler_matches_reference(gold):
    from graphneuralnetwork_amd.pysampler import PyAdjacency, get_layer_adj_nodes
    adjs = {n: PyAdjacency(gold[f"{n}_adj_ptr"], gold[f"{n}_adj_nbr"]) for n in GRAPHS}
    for c, name, L, K, gcn in _cases(gold):
        r = _rng_at(gold[f"case{c}_state0"])
        neigh, center = get_layer_adj_nodes(gold[f"case{c}_nodes"], adjs[name], L, K, gcn, rng=r)
        assert neigh.dtype == torch.int64 and center.dtype == torch.int64
        np.testing.assert_array_equal(neigh.numpy(), gold[f"case{c}_neigh"], err_msg=f"case {c}")
        np.testing.assert_array_equal(center.numpy(), gold[f"case{c}_center"])
        np.testing.assert_array_equal(np.asarray(r.getstate()[1], np.uint32),
                                      gold[f"case{c}_state1"])


def test_global_random_is_consumed_like_the_reference(gold):
    """Default rng = the global ``random`` module: same maps, same state afterwards."""
    from graphneuralnetwork_amd.pysampler import get_layer_adj_nodes
    adj = _adj_lists(gold, "small")
    c = 0
    _, name, L, K, gcn = next(_cases(gold))
    random.setstate((3, tuple(int(w) for w in gold[f"case{c}_state0"]), None))
    neigh, center = get_layer_adj_nodes(gold[f"case{c}_nodes"].tolist(), adj, L, K, gcn)
    np.testing.assert_array_equal(neigh.numpy(), gold[f"case{c}_neigh"])
    np.testing.assert_array_equal(np.asarray(random.getstate()[1], np.uint32),
                                  gold[f"case{c}_state1"])


def test_empty_neighbourhood_raises_like_the_reference(gold):
    from graphneuralnetwork_amd.pysampler import get_layer_adj_nodes
    assert int(gold["empty_raises"]) == 1
    adj = defaultdict(set, {0: {1}, 1: {0}})
    for v in range(2, 6):
        adj[v]  # noqa: B018  (defaultdict: nodes 2..5 exist with no neighbours)
    random.seed(0)
    with pytest.raises(IndexError, match="empty sequence"):
        get_layer_adj_nodes([0, 5], adj, 1, 3, False)
    np.testing.assert_array_equal(np.asarray(random.getstate()[1], np.uint32), gold["empty_state1"])


@pytest.mark.parametrize("seed", range(6))
def test_native_matches_oracle_on_random_graphs(seed):
    """Power-law-ish graphs with hubs above random.sample's set-size switch, 1-3 layers,
    fanouts on both sides of the degrees, gcn on/off, repeated batch nodes."""
    from graphneuralnetwork_amd.pysampler import PyAdjacency, get_layer_adj_nodes
    rs = np.random.default_rng(100 + seed)
    n = int(rs.integers(50, 3000))
    m = int(rs.integers(2 * n, 8 * n))
    src = np.minimum((rs.pareto(1.2, m) * 3).astype(np.int64), n - 1)
    dst = rs.integers(0, n, m)
    ring = np.arange(n)
    src = np.concatenate([ring, src])
    dst = np.concatenate([(ring + 1) % n, dst])
    adj = defaultdict(set)
    for a, b in zip(src.tolist(), dst.tolist()):
        adj[a].add(b)
        adj[b].add(a)
    pa = PyAdjacency.from_pairs(src, dst, n)
    L = int(rs.integers(1, 4))
    K = int(rs.choice([1, 3, 5, 6, 10, 25]))
    gcn = bool(seed % 2)
    B = int(rs.integers(1, min(n, 64)))
    nodes = rs.choice(n, B, replace=False).tolist()
    if B > 3:
        nodes[-1] = nodes[0]
    r1, r2 = random.Random(seed), random.Random(seed)
    try:
        ref = O.sage_layer_adj_nodes(nodes, adj, L, K, gcn, r1)
    except (IndexError, ValueError):
        pytest.skip("configuration the reference itself rejects")
    neigh, center = get_layer_adj_nodes(nodes, pa, L, K, gcn, rng=r2)
    np.testing.assert_array_equal(neigh.numpy(), np.asarray(ref[0]))
    np.testing.assert_array_equal(center.numpy(), np.asarray(ref[1]))
    assert r1.getstate() == r2.getstate()


def test_set_order_matches_cpython():
    """The set-table restatement against CPython itself, incl. > 50,000-entry tables."""
    from graphneuralnetwork_amd import _lib
    lib = _lib.load()
    rng = random.Random(7)

    def run(fn, *arrs):
        arrs = [np.ascontiguousarray(a, np.int64) for a in arrs]
        out = np.empty(max(1, sum(a.size for a in arrs)), np.int64)
        n = ctypes.c_int64()
        args = [x for a in arrs for x in (a.ctypes.data, a.size)]
        assert fn(*args, out.ctypes.data, ctypes.byref(n)) == 0
        return out[: n.value].tolist()

    for t in range(300):
        hi = rng.choice([16, 1000, 10 ** 6, 2 ** 40])
        a = [rng.randrange(hi) for _ in range(rng.randint(0, 500))]
        b = [rng.randrange(hi) for _ in range(rng.randint(0, 500))]
        assert run(lib.gnn_pyset_order, a) == list(set(a))
        assert run(lib.gnn_pyset_union_order, a, b) == list(set(a).union(set(b)))
    a = [rng.randrange(10 ** 8) for _ in range(200_000)]
    b = [rng.randrange(10 ** 8) for _ in range(60_000)]
    assert run(lib.gnn_pyset_order, a) == list(set(a))
    assert run(lib.gnn_pyset_union_order, a, b) == list(set(a).union(set(b)))


@pytest.mark.gpu
def test_collate_fn_on_device(gold):
    """collate_fn: the reference's output tuple, maps bit-exact, rows gathered on the device."""
    from graphneuralnetwork_amd.pysampler import collate_fn
    adj = _adj_lists(gold, "small")
    n = int(gold["small_n"])
    feat = np.random.default_rng(0).standard_normal((n, 24)).astype(np.float32)
    c = 0
    _, name, L, K, gcn = next(_cases(gold))
    r = _rng_at(gold[f"case{c}_state0"])
    col = collate_fn(adj, feat.tolist(), L, K, gcn, False, rng=r)
    nodes = gold[f"case{c}_nodes"].tolist()
    X, y = col(list(zip(nodes, range(len(nodes)))))
    neigh, center = gold[f"case{c}_neigh"], gold[f"case{c}_center"]
    np.testing.assert_array_equal(X[0].cpu().numpy(), feat[center[0]])
    np.testing.assert_array_equal(X[1].cpu().numpy(), center[1:])
    np.testing.assert_array_equal(X[2].cpu().numpy(), feat[neigh[0]])
    np.testing.assert_array_equal(X[3].cpu().numpy(), neigh[1:])
    np.testing.assert_array_equal(y.numpy(), np.arange(len(nodes)))
