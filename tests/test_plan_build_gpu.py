"""The device schedule builders (csrc/plan_build.hip) against the torch builders of graph.py.

gnn_spmm_tasks_build, gnn_column_order and gnn_xcd_hub_plan_build / _fill restate
graph.task_ranges_torch, graph._degree_perm_torch (+ the column rename) and graph.xcd_hub_coo
+ from_coo; every output array must be EQUAL (integer schedules, copied fp32 values), on
ragged graphs with empty rows, single rows and R-MAT hubs, at the bench's cfg2 size too. The
SpMM results through these schedules are pinned against the oracle by test_spmm_gpu.py and
test_fullsize_gpu.py (graph.NATIVE_PLANS is the default path).
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _csr_from_degrees(deg, n_cols, seed):
    from graphneuralnetwork_amd.graph import CsrGraph
    rng = np.random.default_rng(seed)
    deg = np.asarray(deg, np.int64)
    rowptr = np.zeros(deg.size + 1, np.int64)
    np.cumsum(deg, out=rowptr[1:])
    nnz = int(rowptr[-1])
    # power-law columns: hubs at random ids
    hot = rng.permutation(n_cols)
    col = hot[np.minimum((rng.pareto(1.2, nnz) * 3).astype(np.int64), n_cols - 1)]
    val = rng.standard_normal(nnz).astype(np.float32)
    return CsrGraph(torch.from_numpy(rowptr).to(DEV), torch.from_numpy(col.astype(np.int32)).to(DEV),
                    torch.from_numpy(val).to(DEV), deg.size, n_cols)


def _rmat_graph(n, m, seed):
    from graphneuralnetwork_amd.preprocess import gcn_adjacency
    from graphneuralnetwork_amd.rmat import rmat_edges
    s, d = rmat_edges(n, m, seed)
    return gcn_adjacency(torch.from_numpy(s).to(DEV), torch.from_numpy(d).to(DEV), n)


def _ragged_degrees(n, seed, long_every=97):
    rng = np.random.default_rng(seed)
    deg = rng.integers(0, 6, n)
    deg[rng.random(n) < 0.2] = 0
    deg[::long_every] = rng.integers(100, 2000, deg[::long_every].size)
    return deg


# ------------------------------------------------------------------------------ tasks
@pytest.mark.parametrize("deg_kind", ["ragged", "all_short", "all_long", "single", "empty_rows"])
@pytest.mark.parametrize("max_deg,cost", [(128, 256), (1, 1), (5, 7), (0, 3), (4096, 64)])
def test_tasks_native_equals_torch(deg_kind, max_deg, cost):
    from graphneuralnetwork_amd.graph import task_ranges_native, task_ranges_torch
    rng = np.random.default_rng(7)
    deg = {"ragged": _ragged_degrees(5000, 1), "all_short": rng.integers(1, 4, 3000),
           "all_long": rng.integers(200, 300, 500), "single": np.array([3]),
           "empty_rows": np.zeros(1000, np.int64)}[deg_kind]
    g = _csr_from_degrees(deg, 777, 3)
    a = task_ranges_native(g.rowptr, max_deg, cost)
    b = task_ranges_torch(g.rowptr, max_deg, cost)
    assert a.dtype == b.dtype == torch.int32
    assert torch.equal(a, b)


def test_tasks_native_full_size_cfg2():
    """The cfg2 graph's tasks (1M rows) as ops.spmm_forward builds them."""
    from graphneuralnetwork_amd.graph import check_tasks, task_ranges_native, task_ranges_torch
    g = _rmat_graph(1_000_000, 10_000_000, 0)
    for max_deg, cost in ((128, 256), (64, 512)):
        a = task_ranges_native(g.rowptr, max_deg, cost)
        assert torch.equal(a, task_ranges_torch(g.rowptr, max_deg, cost))
        check_tasks(a, g.n_rows)


def test_tasks_capacity_protocol():
    """cap too small: GNN_E_ARG with the count set; null task_row: count only."""
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.graph import task_ranges_torch
    lib = _lib.load()
    g = _csr_from_degrees(_ragged_degrees(3000, 2), 100, 4)
    n = g.n_rows
    want = task_ranges_torch(g.rowptr, 128, 256).numel() // 2
    ws = torch.empty(int(lib.gnn_spmm_tasks_workspace_bytes(n)), dtype=torch.uint8, device=DEV)
    nt = ctypes.c_int64(-1)
    s = _lib.stream_handle(DEV)
    assert lib.gnn_spmm_tasks_build(g.rowptr.data_ptr(), n, 128, 256, None, 0,
                                    ctypes.addressof(nt), ws.data_ptr(), ws.numel(), s) == 0
    assert nt.value == want
    out = torch.full((2 * want,), -7, dtype=torch.int32, device=DEV)
    assert lib.gnn_spmm_tasks_build(g.rowptr.data_ptr(), n, 128, 256, out.data_ptr(), want - 1,
                                    ctypes.addressof(nt), ws.data_ptr(), ws.numel(), s) == -1
    assert nt.value == want and int((out != -7).sum()) == 0
    assert lib.gnn_spmm_tasks_build(g.rowptr.data_ptr(), n, 128, 256, out.data_ptr(), want,
                                    ctypes.addressof(nt), ws.data_ptr(), ws.numel(), s) == 0
    assert torch.equal(out, task_ranges_torch(g.rowptr, 128, 256))
    # cost < 1 and a short workspace are argument errors
    assert lib.gnn_spmm_tasks_build(g.rowptr.data_ptr(), n, 128, 0, None, 0, ctypes.addressof(nt),
                                    ws.data_ptr(), ws.numel(), s) == -1
    assert lib.gnn_spmm_tasks_build(g.rowptr.data_ptr(), n, 128, 256, None, 0,
                                    ctypes.addressof(nt), ws.data_ptr(), 16, s) == -1


# ------------------------------------------------------------------------------ column order
@pytest.mark.parametrize("prefix,tail", [(None, None), (0, None), (10, None), (10, "degree"),
                                         (499, "id"), (500, None), (5000, None)])
@pytest.mark.parametrize("rows", [False, True])
def test_column_order_native_equals_torch(monkeypatch, prefix, tail, rows):
    from graphneuralnetwork_amd import graph as G
    g = _csr_from_degrees(_ragged_degrees(500, 5), 500, 6)  # square; ties in the degrees
    a = G.degree_order(g, rows=rows, prefix=prefix, tail=tail)
    monkeypatch.setattr(G, "NATIVE_PLANS", False)
    b = G.degree_order(g, rows=rows, prefix=prefix, tail=tail)
    assert torch.equal(a.perm, b.perm) and torch.equal(a.inv, b.inv)
    for k in ("rowptr", "col", "val"):
        assert torch.equal(getattr(a.graph, k), getattr(b.graph, k)), k


def test_column_order_native_rmat_and_errors():
    from graphneuralnetwork_amd import _lib
    from graphneuralnetwork_amd.graph import _degree_perm_torch, column_order_native
    g = _rmat_graph(200_000, 2_000_000, 3)
    for prefix in (-1, 4096, 262_144):
        perm, inv, col = column_order_native(g, prefix)
        p2, i2 = _degree_perm_torch(g, None if prefix < 0 else prefix, None)
        assert torch.equal(perm, p2) and torch.equal(inv, i2)
        assert torch.equal(col, inv[g.col.long()].int())
    # a column id outside [0, n_cols) is an argument error
    lib = _lib.load()
    bad = torch.tensor([0, 5, 9], dtype=torch.int32, device=DEV)
    ws = torch.empty(int(lib.gnn_column_order_workspace_bytes(8)), dtype=torch.uint8, device=DEV)
    perm = torch.empty(8, dtype=torch.int64, device=DEV)
    inv = torch.empty_like(perm)
    out = torch.empty_like(bad)
    assert lib.gnn_column_order(bad.data_ptr(), 3, 8, -1, perm.data_ptr(), inv.data_ptr(),
                                out.data_ptr(), ws.data_ptr(), ws.numel(),
                                _lib.stream_handle(DEV)) == -1


# ------------------------------------------------------------------------------ XCD hub plan
def _xcd_pair(monkeypatch, g, k, min_deg, chunk, phases=1, item_k=None, small_item=None):
    from graphneuralnetwork_amd import graph as G
    a = G._build_xcd_hub_plan(g, k, min_deg, chunk, phases, item_k, small_item)
    with monkeypatch.context() as m:
        m.setattr(G, "NATIVE_PLANS", False)
        b = G._build_xcd_hub_plan(g, k, min_deg, chunk, phases, item_k, small_item)
    return a, b


def _assert_same_plan(a, b):
    assert (a is None) == (b is None)
    if a is None:
        return
    assert a.n_items == b.n_items and a.n_pos == b.n_pos
    assert torch.equal(a.item_row, b.item_row)
    for part in ("items", "rest"):
        ga, gb = getattr(a, part), getattr(b, part)
        assert (ga.n_rows, ga.n_cols) == (gb.n_rows, gb.n_cols), part
        for k in ("rowptr", "col", "val"):
            assert torch.equal(getattr(ga, k), getattr(gb, k)), (part, k)


@pytest.mark.parametrize("cfg", [
    dict(k=64, min_deg=16, chunk=8),
    dict(k=64, min_deg=16, chunk=4, phases=2),
    dict(k=256, min_deg=32, chunk=16, item_k=40),
    dict(k=64, min_deg=64, chunk=8, small_item=2),
    dict(k=128, min_deg=16, chunk=128, phases=3, small_item=3),
    dict(k=16, min_deg=100000, chunk=8),  # no row qualifies: no plan
])
def test_xcd_plan_native_equals_torch(monkeypatch, cfg):
    g = _csr_from_degrees(_ragged_degrees(4000, 8, long_every=31), 3000, 9)
    hub = g.hub_plan(cfg["k"])
    assert hub.k == cfg["k"]
    a, b = _xcd_pair(monkeypatch, g, **cfg)
    _assert_same_plan(a, b)
    if cfg["min_deg"] < 1000:
        assert a is not None and a.n_items > 0


def test_xcd_plan_native_equals_torch_cfg2_ordered(monkeypatch):
    """The plan bench.py's cfg2 step runs: the column-ordered 1M-node graph, K = 262144 hub rows
    read in place, XCD_MIN_DEG / XCD_CHUNK defaults."""
    from graphneuralnetwork_amd import ops
    from graphneuralnetwork_amd.graph import degree_order
    g = _rmat_graph(1_000_000, 10_000_000, 0)
    o = degree_order(g, rows=False, prefix=ops.XCD_HUB_ROWS)
    k = ops.xcd_hub_rows_for(g.n_cols, 128)
    a, b = _xcd_pair(monkeypatch, o.graph, k, ops.XCD_MIN_DEG, ops.XCD_CHUNK)
    assert a is not None and a.prefix
    _assert_same_plan(a, b)
