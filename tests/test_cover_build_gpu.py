"""The device cover-exchange builder (csrc/cover_build.hip: gnn_cover_build / _fill /
_send_partials) against the torch restatement in distributed.py.

Every rank of a LocalGroup (ranks as threads on one GPU) builds its CoverExchange twice --
through the C-ABI (distributed.NATIVE_COVER, the default on the device) and through torch ops
-- and every array must be EQUAL: the interior / halo_x / halo_p / send_p CSRs, the send list
and the per-peer counts. Graphs: R-MAT (hub columns, the greedy rule's both outcomes), a
ragged graph with empty rows and a rank without edges, world 1, 2, 3 and 8. The SpMM through
these partitions is compared with the single-GPU SpMM by test_distributed_gpu.py.
"""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rmat(n, m, seed, dev):
    from graphneuralnetwork_amd.preprocess import gcn_normalized_csr
    from graphneuralnetwork_amd.rmat import rmat_edges
    s, d = rmat_edges(n, m, seed)
    return gcn_normalized_csr(s, d, n, device=dev)


def _ragged(n, dev, seed=4):
    from graphneuralnetwork_amd.graph import CsrGraph
    rng = np.random.default_rng(seed)
    deg = rng.integers(0, 7, n)
    deg[: n // 5] = 0                     # the first rank's rows have no edges
    deg[n // 2] = 3000                    # one long row
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(deg, out=rowptr[1:])
    col = rng.integers(0, n, int(rowptr[-1])).astype(np.int32)
    col[rng.random(col.size) < 0.3] = 7  # a hub column
    val = rng.standard_normal(col.size).astype(np.float32)
    return CsrGraph(torch.from_numpy(rowptr).to(dev), torch.from_numpy(col).to(dev),
                    torch.from_numpy(val).to(dev), n, n)


def _build_all(D, g, world, native, bounds=None):
    comm = D.LocalGroup(world)
    parts = [None] * world
    errs = []

    def main(r):
        try:
            comm.bind(r)
            parts[r] = D.build_cover_exchange(g, r, world, group=comm, bounds=bounds)
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            errs.append(e)
            comm._bar.abort()

    old = D.NATIVE_COVER
    D.NATIVE_COVER = native
    try:
        th = [threading.Thread(target=main, args=(r,)) for r in range(world)]
        [t.start() for t in th]
        [t.join() for t in th]
    finally:
        D.NATIVE_COVER = old
    if errs:
        raise errs[0]
    return parts


def _same_csr(a, b, what):
    assert (a.n_rows, a.n_cols) == (b.n_rows, b.n_cols), what
    for k in ("rowptr", "col", "val"):
        x, y = getattr(a, k), getattr(b, k)
        assert x.dtype == y.dtype and torch.equal(x.cpu(), y.cpu()), (what, k)


def _same(pa, pb):
    for r, (a, b) in enumerate(zip(pa, pb)):
        assert a.bounds == b.bounds
        for what in ("interior", "send_p", "halo_x", "halo_p"):
            _same_csr(getattr(a, what), getattr(b, what), (r, what))
        assert torch.equal(a.send_x_idx.cpu(), b.send_x_idx.cpu()), r
        for k in ("send_x_counts", "send_p_counts", "recv_x_counts", "recv_p_counts", "any_x",
                  "any_p"):
            assert getattr(a, k) == getattr(b, k), (r, k)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_cover_native_equals_torch_rmat(dev, world):
    from graphneuralnetwork_amd import distributed as D
    g = _rmat(30000, 300000, 5, dev)
    pa = _build_all(D, g, world, True)
    pb = _build_all(D, g, world, False)
    _same(pa, pb)
    if world > 1:  # both cover kinds occur
        assert sum(p.n_feature_recv for p in pa) > 0 and sum(p.n_partial_recv for p in pa) > 0


def test_cover_native_equals_torch_ragged(dev):
    from graphneuralnetwork_amd import distributed as D
    g = _ragged(5000, dev)
    for world in (2, 5):
        _same(_build_all(D, g, world, True), _build_all(D, g, world, False))
    # explicit bounds with an empty block
    b = torch.tensor([0, 1000, 1000, 5000])
    _same(_build_all(D, g, 3, True, b), _build_all(D, g, 3, False, b))


def test_cover_capi_rejects_bad_bounds(dev):
    import ctypes
    from graphneuralnetwork_amd import _lib
    lib = _lib.load()
    g = _ragged(100, dev)
    ws = torch.empty(int(lib.gnn_cover_workspace_bytes(100, g.nnz, 100, 2)), dtype=torch.uint8,
                     device=dev)
    counts = (ctypes.c_int64 * 10)()
    s = _lib.stream_handle(dev)
    for bad in ([0, 60, 50], [0, 50, 99], [1, 50, 100]):  # descending, short, not from 0
        hb = (ctypes.c_int64 * 3)(*bad)
        assert lib.gnn_cover_build(g.rowptr.data_ptr(), g.col.data_ptr(), 100, ctypes.addressof(hb),
                                   0, 2, ctypes.addressof(counts), ws.data_ptr(), ws.numel(),
                                   s) == -1
    hb = (ctypes.c_int64 * 3)(0, 50, 100)
    assert lib.gnn_cover_build(g.rowptr.data_ptr(), g.col.data_ptr(), 100, ctypes.addressof(hb), 2,
                               2, ctypes.addressof(counts), ws.data_ptr(), ws.numel(), s) == -1
    # a column id outside [0, n_rows) in this rank's rows
    bad_col = g.col.clone()
    bad_col[int(g.rowptr[60])] = 100
    hb = (ctypes.c_int64 * 3)(0, 50, 100)
    assert lib.gnn_cover_build(g.rowptr.data_ptr(), bad_col.data_ptr(), 100, ctypes.addressof(hb),
                               1, 2, ctypes.addressof(counts), ws.data_ptr(), ws.numel(), s) == -1
    # the handshake's partial-row total must match the received edges' slots
    pe_i = torch.tensor([3, 3, 4], dtype=torch.int64, device=dev)
    pe_j = torch.tensor([0, 1, 1], dtype=torch.int64, device=dev)
    pe_v = torch.ones(3, device=dev)
    he = (ctypes.c_int64 * 1)(3)
    sws = torch.empty(int(lib.gnn_cover_send_workspace_bytes(3)), dtype=torch.uint8, device=dev)
    rp = torch.empty(3, dtype=torch.int64, device=dev)
    col = torch.empty(3, dtype=torch.int32, device=dev)
    val = torch.empty(3, device=dev)
    args = (pe_i.data_ptr(), pe_j.data_ptr(), pe_v.data_ptr(), ctypes.addressof(he), 1, 0, 2)
    assert lib.gnn_cover_send_partials(*args, 3, rp.data_ptr(), col.data_ptr(), val.data_ptr(),
                                       sws.data_ptr(), sws.numel(), s) == -1
    assert lib.gnn_cover_send_partials(*args, 2, rp.data_ptr(), col.data_ptr(), val.data_ptr(),
                                       sws.data_ptr(), sws.numel(), s) == 0
    assert rp.cpu().tolist()[:3] == [0, 2, 3] and col.cpu().tolist() == [0, 1, 1]
