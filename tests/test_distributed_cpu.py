"""Edge-cut partition + halo all-to-all-v on gloo (world_size 2 and 3, CPU).

The HIP kernels are replaced by the CPU oracle here (these tests exercise the
partitioning, the send/recv-list negotiation and the exchange); the same
EdgeCutSpmm runs the HIP kernels over RCCL on the GPU box (bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gnn_oracle as O


def _collect(procs, q, n, timeout=600):
    """Results from n workers; fails fast when a worker dies instead of waiting for the timeout."""
    import queue
    import time
    out, t0 = [], time.time()
    while len(out) < n:
        try:
            out.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.time() - t0 > timeout:
                for p in procs:
                    p.kill()
                raise AssertionError(f"worker failed (exit codes {dead}) or timed out")
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cpu_spmm(g, x, bias=None, activation=None, out=None, accumulate=False):
    y = O.spmm_csr(g.rowptr.numpy(), g.col.numpy(), g.val.numpy(), x.numpy(), None)
    if accumulate:
        y = y + out.numpy().astype(np.float64)
    if bias is not None:
        y = y + bias.numpy()
    if activation == "relu":
        y = np.maximum(y, 0)
    out.copy_(torch.from_numpy(y.astype(np.float32)))
    return out


def _cpu_gather(x, idx, out):
    out.copy_(x[idx])
    return out


def _graph(n, seed):
    from graphneuralnetwork_amd.preprocess import gcn_normalized_csr
    from graphneuralnetwork_amd.rmat import rmat_edges
    s, d = rmat_edges(n, 8 * n, seed)
    return gcn_normalized_csr(s, d, n)


def _worker(rank, world, port, n, F, q, kind="gather"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    kind, _, chunks = kind.partition(":")  # "cover:3" = the feature rows in 3 chunked exchanges
    chunks = int(chunks) if chunks else None
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphneuralnetwork_amd.distributed import (EdgeCutSpmm, build_cover_exchange,
                                                        build_cover_exchange_balanced,
                                                        build_partition)
        g = _graph(n, 3)
        if kind in ("cover", "balanced"):
            if kind == "cover":
                part = build_cover_exchange(g, rank, world)
            else:
                part, hist = build_cover_exchange_balanced(g, rank, world)
                assert len(hist) == 3 and min(h[0] for h in hist) <= hist[0][0]
            # cut edges reduced here: halo column entries + partial edges computed for peers
            edges = part.interior.nnz + part.halo_x.nnz + part.send_p.nnz
        else:
            part = build_partition(g, rank, world)
            edges = part.nnz
        X = torch.from_numpy(np.random.default_rng(0).standard_normal((n, F)).astype(np.float32))
        b = torch.arange(F, dtype=torch.float32) / F
        r0, r1 = part.bounds[rank], part.bounds[rank + 1]
        run = EdgeCutSpmm(part, F, "cpu", spmm=_cpu_spmm, gather=_cpu_gather, chunks=chunks)
        if chunks is not None and kind != "gather":
            assert run.chunks == chunks and len(run.halo_x_chunks) == chunks
            assert sum(c.nnz for c in run.halo_x_chunks) == part.halo_x.nnz
        y_t = run(X[r0:r1].contiguous(), b, activation="relu")
        y = y_t.clone()
        # stacked layers: the result fed straight back as x lands in the other buffer
        y2 = run(y_t, b, activation="relu").clone()
        assert torch.equal(y_t, y), "the previous result was overwritten by the next call"
        try:
            run(y_t, b, out=y_t)
            aliased = False
        except ValueError:
            aliased = True
        assert aliased, "x aliasing the output buffer must be rejected"
        q.put((rank, r0, r1, (y.numpy(), y2.numpy()), edges, part.n_halo, part.send_counts,
               part.recv_counts))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind", [(2, "gather"), (3, "gather"), (2, "cover"), (3, "cover"),
                                        (3, "balanced"), (2, "cover:1"), (3, "cover:3"),
                                        (2, "cover:7000")])
def test_edge_cut_matches_single_device(world, kind):
    n, F = 3000, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, F, q, kind))
             for r in range(world)]
    for p in procs:
        p.start()
    res = _collect(procs, q, world, 300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = _graph(n, 3)
    X = np.random.default_rng(0).standard_normal((n, F)).astype(np.float32)
    bias = np.arange(F, dtype=np.float32) / F
    ref = np.maximum(O.spmm_csr(g.rowptr.numpy(), g.col.numpy(), g.val.numpy(), X, bias), 0)
    ref2 = np.maximum(O.spmm_csr(g.rowptr.numpy(), g.col.numpy(), g.val.numpy(),
                                 ref.astype(np.float32), bias), 0)
    res.sort(key=lambda t: t[0])
    covered = 0
    tot_nnz = 0
    sends = {}
    for rank, r0, r1, (y, y2), nnz, n_halo, sc, rc in res:
        np.testing.assert_allclose(y, ref[r0:r1], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(y2, ref2[r0:r1], rtol=1e-4, atol=1e-5)
        covered += r1 - r0
        tot_nnz += nnz
        sends[rank] = (sc, rc)
        assert sum(rc) == n_halo
    assert covered == n and tot_nnz == g.nnz
    for p in range(world):  # what p sends to q is what q receives from p
        for qq in range(world):
            assert sends[p][0][qq] == sends[qq][1][p]


def _blockdiag_worker(rank, world, port, q):
    """Rows of each rank only touch its own columns: no exchange at all (any_x = any_p = False)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphneuralnetwork_amd.distributed import EdgeCutSpmm, build_cover_exchange
        from graphneuralnetwork_amd.graph import from_coo
        n, F = 40, 4
        r = torch.arange(n)
        rows = torch.cat([r, r])
        cols = torch.cat([r, (r + 1) % 20 + (r // 20) * 20])   # two 20-cycles + self loops
        g = from_coo(rows, cols, torch.full((2 * n,), -0.5), n, n)
        part = build_cover_exchange(g, rank, world, bounds=torch.tensor([0, 20, 40]))
        X = torch.from_numpy(np.random.default_rng(2).standard_normal((n, F)).astype(np.float32))
        run = EdgeCutSpmm(part, F, "cpu", spmm=_cpu_spmm, gather=_cpu_gather)
        y = run(X[rank * 20:(rank + 1) * 20].contiguous(), None, activation="relu").clone()
        q.put((rank, part.any_x, part.any_p, y.numpy(), X.numpy()))
    finally:
        dist.destroy_process_group()


def test_cover_exchange_without_cut_edges():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_blockdiag_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(_collect(procs, q, 2, 120), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X = res[0][4]
    for rank, ax, ap, y, _ in res:
        assert not ax and not ap
        rr = np.arange(rank * 20, rank * 20 + 20)
        nxt = (rr + 1) % 20 + (rr // 20) * 20
        ref = np.maximum(-0.5 * (X[rr] + X[nxt]), 0)
        np.testing.assert_allclose(y, ref, rtol=1e-6, atol=1e-6)


def test_weighted_bounds():
    from graphneuralnetwork_amd.distributed import nnz_balanced_bounds, weighted_bounds
    rng = np.random.default_rng(1)
    deg = rng.zipf(1.8, 5000).clip(0, 3000)
    rowptr = torch.from_numpy(np.concatenate([[0], np.cumsum(deg)]))
    for w in (2, 3, 8):
        assert torch.equal(weighted_bounds(rowptr, w), nnz_balanced_bounds(rowptr, w))
    b0 = nnz_balanced_bounds(rowptr, 4).tolist()
    # block 0 three times as costly per edge/row: it shrinks, the others grow
    b1 = weighted_bounds(rowptr, 4, [3.0, 1.0, 1.0, 1.0], b0).tolist()
    assert b1[0] == 0 and b1[-1] == 5000 and b1 == sorted(b1) and b1[1] < b0[1]
    c = np.concatenate([[0], np.cumsum((deg + 1) * np.where(np.arange(5000) < b0[1], 3.0, 1.0))])
    part = [c[b1[k + 1]] - c[b1[k]] for k in range(4)]
    assert max(part) - min(part) <= 2 * (deg.max() + 1) * 3


def test_nnz_balanced_bounds():
    from graphneuralnetwork_amd.distributed import nnz_balanced_bounds
    deg = np.array([1, 1, 100, 1, 1, 1, 50, 1, 1, 1])
    rowptr = torch.from_numpy(np.concatenate([[0], np.cumsum(deg)]))
    b = nnz_balanced_bounds(rowptr, 4).tolist()
    assert b[0] == 0 and b[-1] == 10 and b == sorted(b)


def _cpu_gat_logits(wh, heads, fh, a_src, a_dst):
    el, er = O.gat_logits(wh.numpy(), heads, fh, a_src.numpy(), a_dst.numpy())
    return torch.from_numpy(el.astype(np.float32)), torch.from_numpy(er.astype(np.float32))


def _cpu_gat_aggregate(g, wh, el, er, heads, fh, slope, mode, activation=None):
    out = O.gat_csr(g.rowptr.numpy(), g.col.numpy(), wh.numpy(), el.numpy(), er.numpy(), heads,
                    fh, slope, mode == 1)
    if activation == "elu":
        out = np.where(out > 0, out, np.expm1(np.minimum(out, 0)))
    return torch.from_numpy(out.astype(np.float32))


def _gat_worker(rank, world, port, n, heads, fh, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphneuralnetwork_amd.distributed import EdgeCutGat, build_partition
        g = _graph(n, 4)
        part = build_partition(g, rank, world)
        rng = np.random.default_rng(0)
        Wh = torch.from_numpy((rng.standard_normal((n, heads * fh)) * 0.5).astype(np.float32))
        a_s = torch.from_numpy((rng.standard_normal(heads * fh) * 0.3).astype(np.float32))
        a_d = torch.from_numpy((rng.standard_normal(heads * fh) * 0.3).astype(np.float32))
        r0, r1 = part.bounds[rank], part.bounds[rank + 1]
        layer = EdgeCutGat(part, heads, fh, "cpu", logits=_cpu_gat_logits,
                           aggregate=_cpu_gat_aggregate, gather=_cpu_gather)
        y = layer(Wh[r0:r1].contiguous(), a_s, a_d, 0.2, 0, "elu")
        q.put((rank, r0, r1, y.numpy()))
    finally:
        dist.destroy_process_group()


def test_gat_edge_cut_matches_single_device():
    n, heads, fh, world = 2000, 4, 8, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gat_worker, args=(r, world, port, n, heads, fh, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(_collect(procs, q, world, 300), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = _graph(n, 4)
    rng = np.random.default_rng(0)
    Wh = (rng.standard_normal((n, heads * fh)) * 0.5).astype(np.float32)
    a_s = (rng.standard_normal(heads * fh) * 0.3).astype(np.float32)
    a_d = (rng.standard_normal(heads * fh) * 0.3).astype(np.float32)
    el, er = O.gat_logits(Wh, heads, fh, a_s, a_d)
    ref = O.gat_csr(g.rowptr.numpy(), g.col.numpy(), Wh, el, er, heads, fh, 0.2, False)
    ref = np.where(ref > 0, ref, np.expm1(np.minimum(ref, 0)))
    for rank, r0, r1, y in res:
        np.testing.assert_allclose(y, ref[r0:r1], rtol=1e-5, atol=1e-5)


def _sage_shard_worker(rank, world, port, n_seeds, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from graphneuralnetwork_amd.distributed import all_gather_rows, shard_seeds
        seeds = torch.arange(1000, 1000 + n_seeds, dtype=torch.int64)
        mine = shard_seeds(seeds, rank, world)
        # a stand-in per-seed "embedding" [len, 3] and logits [len, 2] of the shard
        emb = torch.stack([mine.float(), mine.float() * 2, torch.full_like(mine, rank).float()], 1)
        got = all_gather_rows(emb, world)
        got1 = all_gather_rows(mine[:, None] * 10, world)
        q.put((rank, mine.numpy(), got.numpy(), got1.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_seeds", [(2, 7), (3, 8), (3, 2)])
def test_sage_seed_shards_and_gather(world, n_seeds):
    """GraphSAGE data parallelism: shard_seeds splits a batch into contiguous,
    disjoint, order-preserving blocks (empty ones too), and all_gather_rows hands every rank
    the rows of all shards in seed order (gloo, world 2-3)."""
    from graphneuralnetwork_amd.distributed import rank_sample_seed
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sage_shard_worker, args=(r, world, port, n_seeds, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(_collect(procs, q, world, 300), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seeds = np.arange(1000, 1000 + n_seeds)
    np.testing.assert_array_equal(np.concatenate([r[1] for r in res]), seeds)
    sizes = [r[1].size for r in res]
    assert max(sizes) - min(sizes) <= 1
    owner = np.concatenate([np.full(r[1].size, r[0]) for r in res])
    for _, _, got, got1 in res:
        np.testing.assert_array_equal(got[:, 0], seeds)
        np.testing.assert_array_equal(got[:, 2], owner)
        np.testing.assert_array_equal(got1[:, 0], seeds * 10)
    assert len({rank_sample_seed(0, r) for r in range(8)}) == 8


@pytest.mark.parametrize("world,kind", [(3, "cover"), (4, "balanced"), (2, "gather")])
def test_local_group_matches_single_device(world, kind):
    """distributed.LocalGroup (the N ranks as threads of one process, collectives as
    in-memory copies) runs the same builders and EdgeCutSpmm exchange as gloo: the row
    blocks concatenate to the single-device A X + b."""
    import threading
    from graphneuralnetwork_amd import distributed as D
    n, F = 2500, 8
    g = _graph(n, 5)
    comm = D.LocalGroup(world)
    X = torch.from_numpy(np.random.default_rng(1).standard_normal((n, F)).astype(np.float32))
    b = torch.arange(F, dtype=torch.float32) / F
    outs, errs = [None] * world, []

    def rank_main(r):
        try:
            comm.bind(r)
            if kind == "cover":
                part = D.build_cover_exchange(g, r, world, group=comm)
            elif kind == "balanced":
                part, _ = D.build_cover_exchange_balanced(g, r, world, group=comm)
            else:
                part = D.build_partition(g, r, world, group=comm)
            r0, r1 = part.bounds[r], part.bounds[r + 1]
            run = D.EdgeCutSpmm(part, F, "cpu", group=comm, spmm=_cpu_spmm, gather=_cpu_gather)
            outs[r] = (r0, run(X[r0:r1].contiguous(), b).clone())
        except Exception as e:  # noqa: BLE001 -- re-raised in the main thread
            errs.append(e)
            comm._bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    if errs:
        raise errs[0]
    y = torch.cat([o[1] for o in sorted(outs, key=lambda o: o[0])]).numpy()
    ref = O.spmm_csr(g.rowptr.numpy(), g.col.numpy(), g.val.numpy(), X.numpy(), b.numpy())
    np.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())


def test_chunk_layout():
    """chunk_sizes / chunk_major: peer q's n_q rows cut into C contiguous pieces; the
    chunk-major buffer holds piece k of every peer (in peer order) for k = 0..C-1, and the
    permutation visits every row once."""
    from graphneuralnetwork_amd.distributed import chunk_major, chunk_sizes
    counts = [5, 0, 3, 8]
    for C in (1, 2, 3, 9):
        cs = chunk_sizes(counts, C)
        assert [sum(col) for col in zip(*cs)] == counts
        perm = chunk_major(counts, C, "cpu")
        assert sorted(perm.tolist()) == list(range(sum(counts)))
        offs = np.concatenate([[0], np.cumsum(counts)])
        pos = 0
        for k in range(C):
            for q, n in enumerate(counts):
                lo, hi = k * n // C, (k + 1) * n // C
                assert perm[pos:pos + hi - lo].tolist() == list(range(offs[q] + lo, offs[q] + hi))
                pos += hi - lo
